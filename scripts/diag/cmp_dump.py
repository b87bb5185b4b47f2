"""Compare two norm_pool_dump.py outputs bitwise: python scripts/diag/cmp_dump.py a.pt b.pt"""
import sys, torch
a = torch.load(sys.argv[1], weights_only=True); b = torch.load(sys.argv[2], weights_only=True)
for k in a:
    fa, wa = a[k]; fb, wb = b[k]
    print(k, "feats_equal", torch.equal(fa.view(torch.int16), fb.view(torch.int16)), "ws_equal", torch.equal(wa, wb))
