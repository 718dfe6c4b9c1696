"""ORACLE — TEST INFRASTRUCTURE ONLY.

CPU restatement of the reference's hot path (src/videotofaces/detectors/mtcnn.py,
encoders/facenet.py, dupes.py, grouping.py) used as the parity checker by tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg.  The product path
(video-to-faces_amd/) never imports this package.
"""
