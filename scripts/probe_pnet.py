"""Time k_pnet alone (vtf_mtcnn_profile) for several VTF_PNET_DEBUG phase-skip masks."""
import os, sys, subprocess, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) > 1 and sys.argv[1] == 'child':
    sys.path[:0] = [ROOT, os.path.join(ROOT, 'video-to-faces_amd')]
    import torch
    from videotofaces import synth
    from videotofaces.detectors.mtcnn import MTCNN
    fr = torch.from_numpy(synth.make_frames(16, seed=0)).cuda()
    m = MTCNN('cuda:0')
    try:
        m(fr, 5)
    except Exception:
        pass
    m.profile(True)
    for _ in range(3):
        try:
            m(fr, 5)
        except Exception as e:
            pass
    ms, n, fl, f = m.profile(False)
    print(json.dumps({'mask': os.environ.get('VTF_PNET_DEBUG', '0'), 'ms': ms / max(n, 1), 'tflops': fl / max(n, 1) / (ms / max(n, 1) / 1e3) / 1e12}))
else:
    for mask in sys.argv[1:] or ['0', '16', '17', '18', '20', '24', '48', '31', '127']:
        env = dict(os.environ, VTF_PNET_DEBUG=mask)
        out = subprocess.run([sys.executable, __file__, 'child'], env=env, capture_output=True, text=True, timeout=300)
        print(out.stdout.strip().splitlines()[-1] if out.stdout.strip() else out.stderr[-500:], flush=True)
