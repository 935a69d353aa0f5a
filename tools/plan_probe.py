import sys, time, ctypes
sys.path.insert(0, "embodied-one-shot-video-recognition_amd")
import torch
from eosv import engine, arch, synth
for dt in ("f32", "bf16", "f32x3"):
    bb = engine.Backbone("resnet18", dt, 224, 224, max_frames=4096, device=0)
    bb.load_state_dict(synth.synth_state_dict(arch.SPECS["resnet18"], 64, 0))
    x = torch.zeros(8, 3, 224, 224, device="cuda")
    torch.cuda.synchronize(); t0 = time.perf_counter(); bb.forward(x); torch.cuda.synchronize()
    print(dt, "first forward incl. pricing %.3f s" % (time.perf_counter() - t0), flush=True)
    bb.close()
