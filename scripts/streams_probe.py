"""Progress-printing probe of the concurrent batch-slice streams at the bench shape."""
import os, sys, time
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from videomamba_amd.videomamba import PretrainVideoMamba

B = int(sys.argv[1]) if len(sys.argv) > 1 else 336
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
dev = torch.device("cuda", 0)
torch.manual_seed(0)
m = PretrainVideoMamba(depth=32, embed_dim=576, num_frames=16).to(dev, torch.bfloat16).eval()
x = torch.randn(B, 3, 16, 224, 224, device=dev).to(torch.bfloat16)
st = m.allocate_state(B, dtype=torch.bfloat16, device=dev)
print("streams", os.environ.get("VM_BATCH_STREAMS"), "B", B, "slices", m._stream_slices(B, st), flush=True)
with torch.no_grad():
    for i in range(steps):
        t0 = time.perf_counter()
        out = m(x, ssm_state=st)
        torch.cuda.synchronize()
        print(f"step {i}: {(time.perf_counter() - t0) * 1e3:.1f} ms  tok/s {B * 16 * 196 / (time.perf_counter() - t0):.0f}  mem {torch.cuda.max_memory_allocated() / 1e9:.1f} GB", flush=True)
