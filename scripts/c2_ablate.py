"""c2 ablation (measurement only, never the reported number): python scripts/c2_ablate.py MODE [bench args]
MODE base: bench.py as is; noenc: every FaceNet encode_crops returns zeros without launching anything
(the detector work alone) -- the difference is what the encoder costs the 4-lane pipeline."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'video-to-faces_amd')]
mode = sys.argv[1]
sys.argv = [os.path.join(ROOT, 'bench.py')] + sys.argv[2:]
import bench  # noqa: E402

if mode == 'noenc':
    import torch
    from videotofaces.encoders.facenet import InceptionResnetV1

    def _zero(self, frames_dev, crops):
        n = crops.shape[0] if hasattr(crops, 'shape') else len(crops)
        return torch.zeros((n, 512), dtype=torch.float32, device=frames_dev.device)
    InceptionResnetV1.encode_crops = _zero
bench.main(sys.argv[1:])
