"""video-to-faces on MI355X: drop-in for the reference package ``videotofaces``.

The public API (``video_to_faces``) and the plugin surface (``get_detector_model``,
``get_encoder_model``, grouping functions) mirror src/videotofaces/; the compute runs in
libvtf_hip.so (hand-written HIP for gfx950).
"""


def video_to_faces(*args, **kwargs):
    from .main import video_to_faces as _v
    return _v(*args, **kwargs)
