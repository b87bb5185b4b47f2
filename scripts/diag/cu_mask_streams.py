"""Sub-batch streams with CU masks (hipExtStreamCreateWithCUMask): each half of the batch
on its own set of CUs, against the product's unmasked streams (first at high priority).
B = 896 M-16f stateful chunk, interleaved rounds:
    python scripts/diag/cu_mask_streams.py"""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from videomamba_amd import videomamba as V  # noqa: E402

dev = torch.device("cuda", 0)
torch.manual_seed(0)
model = V.PretrainVideoMamba(depth=32, embed_dim=576, num_frames=16, pool_type="cls+avg")
model = model.to(device=dev, dtype=torch.bfloat16).eval()
B = 896
g = torch.Generator(device=dev).manual_seed(1000)
x = torch.randn(B, 3, 16, 224, 224, device=dev, generator=g).to(torch.bfloat16)
st = model.allocate_state(B, dtype=torch.bfloat16, device=dev)
key = (dev.type, dev.index)
cus = torch.cuda.get_device_properties(dev).multi_processor_count
hip = ctypes.CDLL("libamdhip64.so")
hip.hipExtStreamCreateWithCUMask.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint32,
                                             ctypes.POINTER(ctypes.c_uint32)]


def masked(bits):
    words = (cus + 31) // 32
    m = (ctypes.c_uint32 * words)()
    for b in bits:
        m[b // 32] |= 1 << (b % 32)
    s = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), words, m)
    assert rc == 0, rc
    return torch.cuda.ExternalStream(s.value, device=dev)


allc = list(range(cus))
modes = {
    "product": V._side_streams(dev, 2),
    "halves": [masked(range(0, cus // 2)), masked(range(cus // 2, cus))],
    "even_odd": [masked(range(0, cus, 2)), masked(range(1, cus, 2))],
    "all_vs_half": [masked(allc), masked(range(0, cus, 2))],
    "all_vs_3q": [masked(allc), masked([c for c in allc if c % 4 != 3])],
}
print(json.dumps({"cus": cus}), flush=True)
with torch.no_grad():
    ref = None
    for mode, ss in modes.items():
        V._SIDE_STREAMS.by_device = {key: ss}  # this thread's side streams
        fresh = model.allocate_state(B, dtype=torch.bfloat16, device=dev)
        out = model(x, ssm_state=fresh, temporal_pos_offset=0)[1].float()
        del fresh
        if ref is None:
            ref = out.clone()
        print(json.dumps({"mode": mode, "pool_bitwise_equal_product": bool(torch.equal(out, ref))}),
              flush=True)
    for r in range(2):
        for mode, ss in modes.items():
            V._SIDE_STREAMS.by_device = {key: ss}  # this thread's side streams
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(3):
                model(x, ssm_state=st, temporal_pos_offset=0)
            torch.cuda.synchronize()
            print(json.dumps({"round": r, "mode": mode,
                              "ms_per_step": round((time.perf_counter() - t0) / 3 * 1e3, 2)}),
                  flush=True)
