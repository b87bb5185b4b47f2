"""GPU parity: HIP kernels (through the C ABI) vs the reference fixtures and the oracle.

Tolerances (stated per check):
* fp32 kernels vs fixtures / oracle: 1e-4 abs+rel (exp2 with folded log2(e), FMA order).
* bf16 outputs: 2e-2 abs+rel (one bf16 ulp is 2^-8 relative; the reference rounds at
  the same points, so differences are single-ulp flips of values computed in fp32).
* states are fp32 inside the kernels: 1e-4 even for bf16 models (1e-2 when stored bf16).
"""

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import load_golden
from oracle import videomamba_oracle as orc
from videomamba_amd import kernels as K

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True, scope="module")
def _gpu():
    assert torch.cuda.is_available(), "gpu-marked tests need a HIP device"


def _t(npz, key, dtype=torch.float32, dev=DEV):
    return torch.from_numpy(npz[key].copy()).to(dtype).to(dev)


def _close(a, b, tol):
    torch.testing.assert_close(a.float().cpu(), b.float().cpu(), rtol=tol, atol=tol)


SCAN, SCAN_META = load_golden("scan_cases.npz")


@pytest.mark.parametrize("name", sorted(SCAN_META))
def test_scan_matches_reference_fixture(name):
    meta = SCAN_META[name]
    dt = torch.bfloat16 if meta["dtype"] == "bfloat16" else torch.float32
    g = lambda k, d=dt: _t(SCAN, f"{name}/{k}", d)  # noqa: E731
    has = lambda k: f"{name}/{k}" in SCAN.files  # noqa: E731
    out, last = K.selective_scan_fn(
        g("u"), g("delta"), g("A", torch.float32), g("B"), g("C"),
        D=g("D", torch.float32) if has("D") else None, z=g("z") if has("z") else None,
        delta_bias=g("delta_bias", torch.float32) if has("delta_bias") else None,
        delta_softplus=meta["softplus"],
        initial_state=g("initial_state", torch.float32) if has("initial_state") else None,
        return_last_state=True)
    assert out.dtype == dt and last.dtype == torch.float32
    _close(out, g("out", torch.float32), 1e-4 if dt == torch.float32 else 2e-2)
    _close(last, g("last_state", torch.float32), 1e-4)


def _rand_scan(Bz, D, L, N, dt, seed, h0=True):
    g = torch.Generator().manual_seed(seed)
    u = torch.randn(Bz, D, L, generator=g)
    delta = 0.5 * torch.randn(Bz, D, L, generator=g) - 1.0
    A = -torch.exp(torch.log(torch.arange(1, N + 1).float()).repeat(D, 1) + 0.1 * torch.randn(D, N, generator=g))
    Bm = torch.randn(Bz, N, L, generator=g)
    Cm = torch.randn(Bz, N, L, generator=g)
    Dv = torch.randn(D, generator=g)
    z = torch.randn(Bz, D, L, generator=g)
    bias = 0.1 * torch.randn(D, generator=g)
    init = torch.randn(Bz, D, N, generator=g) if h0 else None
    return [t.to(dt) if t is not None and i in (0, 1, 3, 4, 6) else t
            for i, t in enumerate((u, delta, A, Bm, Cm, Dv, z, bias, init))]


_ORACLE_CACHE = {}


def _oracle_scan(Bz, D, L, N):
    key = (Bz, D, L, N)
    if key not in _ORACLE_CACHE:
        u, delta, A, Bm, Cm, Dv, z, bias, init = _rand_scan(Bz, D, L, N, torch.float32, 11 + L)
        _ORACLE_CACHE[key] = orc.selective_scan(u, delta, A, Bm, Cm, Dv, z, bias, True, init, True)
    return _ORACLE_CACHE[key]


SCAN_VARIANTS = ["0", "1", "5", "6", "13", "14", "15", "16", "17", "18", "19",
                 "30", "31", "32", "33", "34", "35", "36", "37"]  # 30-35: v5 with the states split over waves


@pytest.fixture(params=SCAN_VARIANTS)
def scan_variant(request, monkeypatch):
    """Every scan kernel variant (VM_SCAN_VARIANT, read per launch) must pass parity."""
    monkeypatch.setenv("VM_SCAN_VARIANT", request.param)
    return request.param


@pytest.mark.parametrize("Bz,D,L,N", [(1, 40, 3137, 16),    # several blocks, ragged dim
                                      (64, 72, 300, 16),    # many channels
                                      (2, 24, 777, 8), (3, 20, 100, 4), (1, 8, 0, 16),
                                      (1, 16, 9000, 16)])   # > 8 waves x 512 steps
def test_scan_matches_oracle_random(Bz, D, L, N, scan_variant):
    u, delta, A, Bm, Cm, Dv, z, bias, init = _rand_scan(Bz, D, L, N, torch.float32, 11 + L)
    ref_y, ref_h = _oracle_scan(Bz, D, L, N)
    cu = lambda t: None if t is None else t.to(DEV)  # noqa: E731
    y, h = K.selective_scan_fn(cu(u), cu(delta), cu(A), cu(Bm), cu(Cm), cu(Dv), cu(z), cu(bias),
                               True, True, cu(init))
    _close(y, ref_y, 1e-4)
    _close(h, ref_h, 1e-4)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_scan_full_size_chunked_equals_full(dt, scan_variant):
    """Size-independent property at the north-star size (D_inner=1152, L=3137): a scan
    split at any point with the carried fp32 state equals the full-sequence scan."""
    u, delta, A, Bm, Cm, Dv, z, bias, _ = _rand_scan(1, 1152, 3137, 16, dt, 5, h0=False)
    cu = lambda t: t.to(DEV)  # noqa: E731
    args = [cu(t) for t in (u, delta, A, Bm, Cm, Dv, z, bias)]
    y_full, h_full = K.selective_scan_fn(*args[:6], z=args[6], delta_bias=args[7],
                                         delta_softplus=True, return_last_state=True)
    s = 1000
    sl = lambda t, a, b: t[..., a:b].contiguous()  # noqa: E731
    y1, h1 = K.selective_scan_fn(sl(args[0], 0, s), sl(args[1], 0, s), args[2], sl(args[3], 0, s),
                                 sl(args[4], 0, s), args[5], z=sl(args[6], 0, s), delta_bias=args[7],
                                 delta_softplus=True, return_last_state=True)
    y2, h2 = K.selective_scan_fn(sl(args[0], s, None), sl(args[1], s, None), args[2],
                                 sl(args[3], s, None), sl(args[4], s, None), args[5],
                                 z=sl(args[6], s, None), delta_bias=args[7], delta_softplus=True,
                                 return_last_state=True, initial_state=h1)
    y_ch = torch.cat([y1, y2], dim=-1)
    rel = ((y_ch.float() - y_full.float()).norm() / y_full.float().norm()).item()
    assert rel < (1e-5 if dt == torch.float32 else 1e-3), rel
    assert ((h2 - h_full).norm() / h_full.norm()).item() < 1e-5
    assert torch.isfinite(y_full.float()).all()


def _tm(t):
    """Same (b, d, l) values stored token-major (unit channel stride)."""
    return None if t is None else t.transpose(1, 2).contiguous().transpose(1, 2)


@pytest.mark.parametrize("segments", ["0", "1", "3", "64", "256"])
@pytest.mark.parametrize("Bz,D,L,N", [(1, 40, 3137, 16),    # ragged channel group
                                      (64, 72, 300, 16),    # many rows
                                      (2, 24, 777, 8), (3, 20, 100, 4), (1, 8, 0, 16),
                                      (1, 130, 9000, 16), (2, 64, 31, 16)])
def test_scan_token_major_matches_oracle(Bz, D, L, N, segments, monkeypatch):
    """Token-major operands take the channel-per-lane kernels: single pass, and the
    segmented summary/carry/final form (VM_SCAN_SEGMENTS forces the segment count;
    "0" = the cost model's choice)."""
    monkeypatch.setenv("VM_SCAN_SEGMENTS", segments)
    u, delta, A, Bm, Cm, Dv, z, bias, init = _rand_scan(Bz, D, L, N, torch.float32, 11 + L)
    ref_y, ref_h = _oracle_scan(Bz, D, L, N)
    cu = lambda t: None if t is None else _tm(t.to(DEV))  # noqa: E731
    y, h = K.selective_scan_fn(cu(u), cu(delta), A.to(DEV), cu(Bm), cu(Cm), Dv.to(DEV), cu(z),
                               bias.to(DEV), True, True, init.to(DEV))
    assert y.stride(1) == 1 or D == 1
    _close(y, ref_y, 1e-4)
    _close(h, ref_h, 1e-4)


@pytest.mark.parametrize("segments", ["0", "1", "16", "256"])
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_scan_token_major_full_size_chunked_equals_full(dt, segments, monkeypatch):
    """North-star size (D_inner=1152, L=3137), token-major: split scan with the carried
    fp32 state == full scan; and == the channel-major kernels."""
    monkeypatch.setenv("VM_SCAN_SEGMENTS", segments)
    u, delta, A, Bm, Cm, Dv, z, bias, _ = _rand_scan(2, 1152, 3137, 16, dt, 5, h0=False)
    cm = [t.to(DEV) for t in (u, delta, A, Bm, Cm, Dv, z, bias)]
    tm = [_tm(t) if t.dim() == 3 else t for t in cm]
    y_full, h_full = K.selective_scan_fn(*tm[:6], z=tm[6], delta_bias=tm[7],
                                         delta_softplus=True, return_last_state=True)
    y_cm, h_cm = K.selective_scan_fn(*cm[:6], z=cm[6], delta_bias=cm[7],
                                     delta_softplus=True, return_last_state=True)
    tol = 1e-5 if dt == torch.float32 else 1e-3
    rel = lambda a, b: ((a.float() - b.float()).norm() / b.float().norm()).item()  # noqa: E731
    assert rel(y_full, y_cm) < tol and rel(h_full, h_cm) < 1e-5
    s = 1000
    sl = lambda t, a, b: _tm(t[..., a:b])  # noqa: E731
    y1, h1 = K.selective_scan_fn(sl(cm[0], 0, s), sl(cm[1], 0, s), cm[2], sl(cm[3], 0, s),
                                 sl(cm[4], 0, s), cm[5], z=sl(cm[6], 0, s), delta_bias=cm[7],
                                 delta_softplus=True, return_last_state=True)
    y2, h2 = K.selective_scan_fn(sl(cm[0], s, None), sl(cm[1], s, None), cm[2],
                                 sl(cm[3], s, None), sl(cm[4], s, None), cm[5],
                                 z=sl(cm[6], s, None), delta_bias=cm[7], delta_softplus=True,
                                 return_last_state=True, initial_state=h1)
    assert rel(torch.cat([y1, y2], dim=-1), y_full) < tol
    assert rel(h2, h_full) < 1e-5
    assert torch.isfinite(y_full.float()).all()


@pytest.mark.parametrize("cpl", ["1", "2"])
@pytest.mark.parametrize("segments", ["1", "5"])
@pytest.mark.parametrize("Bz,D,L", [(2, 128, 777), (3, 200, 64), (1, 1152, 3137), (2, 64, 9)])
def test_scan_token_major_bf16_channel_pairs(Bz, D, L, segments, cpl, monkeypatch):
    """bf16 token-major scan with B/C as scalar loads: one channel per lane (cpl=1) and the
    two-adjacent-channels-per-lane kernel (cpl=2, forced), single pass and segmented, vs the
    oracle on the same bf16 inputs (one bf16 rounding of the output) and vs the
    channel-major kernel."""
    monkeypatch.setenv("VM_SCAN_SEGMENTS", segments)
    monkeypatch.setenv("VM_SCAN_CPL", cpl)
    u, delta, A, Bm, Cm, Dv, z, bias, init = _rand_scan(Bz, D, L, 16, torch.bfloat16, 7 + L)
    ref_y, ref_h = orc.selective_scan(u.float(), delta.float(), A, Bm.float(), Cm.float(), Dv,
                                      z.float(), bias, True, init, True)
    cm = [t.to(DEV) if t is not None else None for t in (u, delta, A, Bm, Cm, Dv, z, bias, init)]
    y, h = K.selective_scan_fn(_tm(cm[0]), _tm(cm[1]), cm[2], _tm(cm[3]), _tm(cm[4]), cm[5],
                               _tm(cm[6]), cm[7], True, True, cm[8])
    _close(y, ref_y, 2e-2)
    _close(h, ref_h, 1e-4)
    y_cm, h_cm = K.selective_scan_fn(*cm[:7], cm[7], True, True, cm[8])
    rel = ((y.float() - y_cm.float()).norm() / y_cm.float().norm()).item()
    assert rel < 5e-3, rel
    assert ((h - h_cm).norm() / h_cm.norm()).item() < 1e-5


@pytest.mark.parametrize("segments", ["0", "4"])
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("Bz,D,L", [(2, 128, 1501), (1, 192, 3137), (3, 64, 13)])
def test_scan_mixer_layout_matches_oracle(Bz, D, L, dt, segments, monkeypatch):
    """The token-major mixer's exact operand layout (mamba_simple._forward_padded_tm):
    u / delta / y rows (B*Lp, D) with Lp = round_up(L, 8) and zeroed padding rows, z the
    second half of xz rows (B*Lp, 2D), B and C adjacent columns of one x_dbl row
    (B*Lp, R + 2N) — the one-scalar-load B/C form — and an in-place stateful h.  Covers the
    unclamped main loop, the clamped tail and the padded-row zeroing, vs the oracle."""
    monkeypatch.setenv("VM_SCAN_SEGMENTS", segments)
    N, R = 16, 8
    E = R + 2 * N
    Lp = (L + 7) // 8 * 8
    n = Bz * Lp
    u, delta, A, Bm, Cm, Dv, z, bias, init = _rand_scan(Bz, D, L, N, dt, 31 + L)
    ref_y, ref_h = orc.selective_scan(u.float(), delta.float(), A, Bm.float(), Cm.float(), Dv,
                                      z.float(), bias, True, init, True)
    rows = lambda t: t.transpose(1, 2)  # noqa: E731  (b, d, l) -> (b, l, d)
    U = torch.zeros(Bz, Lp, D, dtype=dt)
    DL = torch.zeros(Bz, Lp, D, dtype=dt)
    XZ = torch.zeros(Bz, Lp, 2 * D, dtype=dt)
    XD = torch.zeros(Bz, Lp, E, dtype=dt)
    U[:, :L], DL[:, :L], XZ[:, :L, D:] = rows(u), rows(delta), rows(z)
    XD[:, :L, R:R + N], XD[:, :L, R + N:] = rows(Bm), rows(Cm)
    U, DL, XZ, XD = (t.reshape(n, -1).to(DEV) for t in (U, DL, XZ, XD))
    y = torch.full((n, D), 7.0, dtype=dt, device=DEV)  # padding rows must come back 0
    h = init.to(DEV).contiguous()
    s_u, s_z, s_bc = (Lp * D, 1, D), (Lp * 2 * D, 1, 2 * D), (Lp * E, 1, E)
    K.scan_raw(U, s_u, DL, s_u, A.to(DEV).contiguous(), XD[:, R:R + N], s_bc, XD[:, R + N:],
               s_bc, Dv.to(DEV), XZ[:, D:], s_z, bias.to(DEV), True, h, (D * N, N), h,
               (D * N, N), y, s_u, Lp, Bz, D, L, N, K.dtype_code(dt),
               torch.cuda.current_stream().cuda_stream)
    y = y.view(Bz, Lp, D)
    _close(y[:, :L].transpose(1, 2), ref_y, 1e-4 if dt == torch.float32 else 2e-2)
    assert not y[:, L:].float().abs().any()
    _close(h, ref_h, 1e-4)


def test_scan_token_major_inplace_bf16_state():
    u, delta, A, Bm, Cm, Dv, z, bias, init = _rand_scan(2, 16, 50, 16, torch.float32, 3)
    st = init.to(DEV).to(torch.bfloat16)
    ref = init.to(torch.bfloat16).float()
    ref_y, ref_h = orc.selective_scan(u, delta, A, Bm, Cm, Dv, z, bias, True, ref, True)
    cu = lambda t: _tm(t.to(DEV))  # noqa: E731
    y, h = K.selective_scan_fn(cu(u), cu(delta), A.to(DEV), cu(Bm), cu(Cm), Dv.to(DEV), cu(z),
                               bias.to(DEV), True, True, st, last_state_out=st)
    assert h is st and h.dtype == torch.bfloat16
    _close(y, ref_y, 1e-4)
    _close(h, ref_h, 1e-2)


def test_scan_inplace_state_alias_and_bf16_state():
    u, delta, A, Bm, Cm, Dv, z, bias, init = _rand_scan(2, 16, 50, 16, torch.float32, 3)
    cu = lambda t: t.to(DEV)  # noqa: E731
    st = cu(init).to(torch.bfloat16)
    ref = init.to(torch.bfloat16).float()
    _, ref_h = orc.selective_scan(u, delta, A, Bm, Cm, Dv, z, bias, True, ref, True)
    _, h = K.selective_scan_fn(cu(u), cu(delta), cu(A), cu(Bm), cu(Cm), cu(Dv), cu(z), cu(bias),
                               True, True, st, last_state_out=st)
    assert h is st and h.dtype == torch.bfloat16
    _close(h, ref_h, 1e-2)


# ------------------------------------------------------------------ conv / norm / step
@pytest.mark.parametrize("with_state", [False, True])
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("L,W", [(37, 4), (3, 4), (1, 4), (16, 2)])
def test_conv1d_matches_oracle(with_state, dt, L, W):
    g = torch.Generator().manual_seed(L * 10 + W)
    x = torch.randn(3, 20, L, generator=g).to(dt)
    w = torch.randn(20, W, generator=g)
    b = torch.randn(20, generator=g)
    cs = torch.randn(3, 20, W, generator=g).to(dt) if with_state else None
    ref, ref_state = orc.causal_conv1d(x, w, b, True, cs)
    out, st = K.causal_conv1d_fn(x.to(DEV), w.to(DEV), b.to(DEV), "silu",
                                 conv_state=None if cs is None else cs.to(DEV),
                                 return_conv_state=True)
    tol = 1e-5 if dt == torch.float32 else 1e-2
    _close(out, ref, tol)
    _close(st, ref_state, 0)


@pytest.mark.parametrize("cols", [16, 100, 192, 576])
@pytest.mark.parametrize("is_rms", [True, False])
@pytest.mark.parametrize("xdt,rdt", [(torch.bfloat16, torch.float32), (torch.float32, None),
                                     (torch.bfloat16, None)])
def test_add_norm_matches_oracle(cols, is_rms, xdt, rdt):
    g = torch.Generator().manual_seed(cols)
    x = torch.randn(37, cols, generator=g).to(xdt)
    res = torch.randn(37, cols, generator=g).to(rdt) if rdt is not None else None
    w = torch.randn(cols, generator=g)
    b = None if is_rms else torch.randn(cols, generator=g)
    ry, rr = orc.add_norm(x, res, w, b, 1e-5, True, True, is_rms)
    fn = K.rms_norm_fn if is_rms else K.layer_norm_fn
    y, r = fn(x.to(DEV), w.to(DEV), None if b is None else b.to(DEV),
              residual=None if res is None else res.to(DEV), prenorm=True,
              residual_in_fp32=True, eps=1e-5)
    assert y.dtype == xdt and r.dtype == rr.dtype
    _close(y, ry, 1e-5 if xdt == torch.float32 else 1e-2)
    _close(r, rr, 1e-6)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_one_token_steps_match_oracle(dt):
    g = torch.Generator().manual_seed(9)
    Bz, D, N, W = 3, 24, 16, 4
    st = torch.randn(Bz, D, N, generator=g)
    x = torch.randn(Bz, D, generator=g).to(dt)
    dtv = torch.randn(Bz, D, generator=g).to(dt)
    A = -torch.rand(D, N, generator=g) * 4
    Bm = torch.randn(Bz, N, generator=g).to(dt)
    Cm = torch.randn(Bz, N, generator=g).to(dt)
    Dv = torch.randn(D, generator=g)
    z = torch.randn(Bz, D, generator=g).to(dt)
    bias = torch.randn(D, generator=g)
    st_ref = st.clone()
    y_ref = orc.selective_state_update(st_ref, x, dtv, A, Bm, Cm, Dv, z, bias, True)
    st_g = st.to(DEV)
    y = K.selective_state_update(st_g, x.to(DEV), dtv.to(DEV), A.to(DEV), Bm.to(DEV),
                                 Cm.to(DEV), Dv.to(DEV), z.to(DEV), bias.to(DEV), True)
    tol = 1e-5 if dt == torch.float32 else 1e-2
    _close(y, y_ref, tol)
    _close(st_g, st_ref, 1e-5)
    cs = torch.randn(Bz, D, W, generator=g).to(dt)
    w = torch.randn(D, W, generator=g)
    cb = torch.randn(D, generator=g)
    cs_ref = cs.clone()
    o_ref = orc.causal_conv1d_update(x, cs_ref, w, cb, True)
    cs_g = cs.to(DEV)
    o = K.causal_conv1d_update(x.to(DEV), cs_g, w.to(DEV), cb.to(DEV), "silu")
    _close(o, o_ref, tol)
    _close(cs_g, cs_ref, 0)


def _patch_oracle(video, w, b, spos, tpos, kt, dt):
    pe = F.conv3d(video.float(), w.float(), b.float(), stride=(kt, w.shape[-2], w.shape[-1])).to(dt)
    Bz, C, Tt, gh, gw = pe.shape
    tok = pe.permute(0, 2, 3, 4, 1).reshape(Bz, Tt, gh * gw, C)
    tok = (tok + spos.to(dt).unsqueeze(0).unsqueeze(0)).to(dt)
    tok = (tok + tpos.to(dt).unsqueeze(0).unsqueeze(2)).to(dt)
    return tok.reshape(Bz, Tt * gh * gw, C)


@pytest.mark.parametrize("dt,Bz,T,H,W,P,kt,C", [
    (torch.bfloat16, 2, 4, 224, 224, 16, 1, 576),   # MFMA path, VideoMamba-M geometry
    (torch.bfloat16, 1, 4, 64, 48, 16, 2, 192),     # MFMA path, tubelet 2, non-square
    (torch.float32, 2, 4, 8, 8, 4, 1, 16),          # generic path (reference test model)
    (torch.bfloat16, 1, 2, 12, 12, 4, 1, 40),       # generic path, bf16
])
def test_patch_embed_matches_oracle(dt, Bz, T, H, W, P, kt, C):
    g = torch.Generator().manual_seed(H + C)
    video = torch.randn(Bz, 3, T, H, W, generator=g).to(dt)
    w = (0.02 * torch.randn(C, 3, kt, P, P, generator=g)).to(dt)
    b = torch.randn(C, generator=g).to(dt)
    hw = (H // P) * (W // P)
    spos = (0.02 * torch.randn(hw, C, generator=g)).to(dt)
    tpos = (0.02 * torch.randn(T // kt, C, generator=g)).to(dt)
    ref = _patch_oracle(video, w, b, spos, tpos, kt, dt)
    out = torch.empty(Bz, ref.shape[1] + 3, C, dtype=dt, device=DEV)
    K.patch_embed(video.to(DEV), w.to(DEV), b.to(DEV), spos.to(DEV), tpos.to(DEV), out, 2,
                  out.stride(0))
    _close(out[:, 2:2 + ref.shape[1]], ref, 1e-5 if dt == torch.float32 else 2e-2)


@pytest.mark.parametrize("Bz,T,H,W,kt,C", [(2, 4, 224, 224, 1, 576), (1, 4, 64, 48, 2, 192),
                                           (6, 32, 224, 224, 1, 192)])  # >= 32768 tokens
def test_patch_embed_wide_tile_matches_small_tile_bitwise(Bz, T, H, W, kt, C, monkeypatch):
    """The 64x192-tile and the LDS-staged 128x192-tile kernels (16x16 patches, embed % 192
    == 0) accumulate in the same k order as the 64x64-tile kernel and round at the same
    points: identical bits."""
    g = torch.Generator().manual_seed(7 + C)
    bf = torch.bfloat16
    video = torch.randn(Bz, 3, T, H, W, generator=g).to(bf).to(DEV)
    w = (0.02 * torch.randn(C, 3, kt, 16, 16, generator=g)).to(bf).to(DEV)
    b = torch.randn(C, generator=g).to(bf).to(DEV)
    hw = (H // 16) * (W // 16)
    spos = (0.02 * torch.randn(hw, C, generator=g)).to(bf).to(DEV)
    tpos = (0.02 * torch.randn(T // kt, C, generator=g)).to(bf).to(DEV)
    outs = []
    for kern in ("0", "1", "2"):
        monkeypatch.setenv("VM_PATCH_KERNEL", kern)
        out = torch.zeros(Bz, (T // kt) * hw + 1, C, dtype=bf, device=DEV)
        K.patch_embed(video, w, b, spos, tpos, out, 1, out.stride(0))
        outs.append(out)
    assert torch.equal(outs[0], outs[1])
    assert torch.equal(outs[2], outs[1])


def test_conv_proj_fused_dt_matches_split_bitwise(monkeypatch):
    """conv_proj with dt_proj inside (default) and as its own kernel (VM_CONV_PROJ_SPLIT=1)
    give identical mixer outputs and states (token-major bf16 mixer, stateful chunks)."""
    from videomamba_amd.mamba_simple import Mamba
    monkeypatch.setenv("VM_MIXER_LAYOUT", "tm")
    torch.manual_seed(3)
    m = Mamba(d_model=64, d_state=16, d_conv=4, expand=2, layer_idx=0).to(DEV, torch.bfloat16)
    x = torch.randn(3, 301, 64, device=DEV).to(torch.bfloat16)
    res = []
    for split in ("0", "1"):
        monkeypatch.setenv("VM_CONV_PROJ_SPLIT", split)
        with torch.no_grad():
            o1, (c1, s1) = m(x[:, :150], return_state=True)
            o2, (c2, s2) = m(x[:, 150:], state=(c1, s1.clone()), return_state=True)
        res.append((o1, c1, o2, c2, s2))
    for a, b in zip(*res):
        assert torch.equal(a, b)


@pytest.mark.parametrize("split", ["0", "1"])
def test_conv_proj_delta_softplus_epilogue(split, monkeypatch):
    """conv_proj's dt epilogue with dt_softplus: delta = softplus(float(bf16(dt)) + bias)
    rounded to bf16, against torch's fp64 softplus applied to the same kernel's plain dt
    output (one bf16 rounding apart: <= 1 ulp = 2^-8 relative).  u and x_dbl unchanged
    (bitwise); fused and split dt_proj forms both.  Includes a stateful first chunk."""
    from videomamba_amd.mamba_simple import Mamba
    monkeypatch.setenv("VM_CONV_PROJ_SPLIT", split)
    torch.manual_seed(5)
    m = Mamba(d_model=96, d_state=16, d_conv=4, expand=2, layer_idx=0).to(DEV, torch.bfloat16)
    Dm, E, R, W = m.d_inner, m.dt_rank + 2 * m.d_state, m.dt_rank, m.d_conv
    Bsz, L = 3, 301
    Lp = (L + 7) // 8 * 8
    n = Bsz * Lp
    xz = torch.randn(n, 2 * Dm, device=DEV).to(torch.bfloat16)
    cs = torch.randn(Bsz, Dm, W, device=DEV).to(torch.bfloat16)
    A, Dv, bias, cw, cb = m._fp32_params()
    bias = bias + torch.linspace(-12.0, 8.0, Dm, device=DEV)  # reach both softplus branches
    wx_pad, wdt_pad = m._padded_proj_weights()
    stream = torch.cuda.current_stream().cuda_stream
    outs = []
    for sp in (False, True):
        u = torch.empty(n, Dm, device=DEV, dtype=torch.bfloat16)
        xd = torch.empty(n, E, device=DEV, dtype=torch.bfloat16)
        dt = torch.empty(n, Dm, device=DEV, dtype=torch.bfloat16)
        K.conv_proj_raw(xz, (Lp * 2 * Dm, 2 * Dm), cw, cb, cs, (cs.stride(0), cs.stride(1)),
                        None, (0, 0), wx_pad, E, wdt_pad, R, u, (Lp * Dm, Dm), xd, (Lp * E, E),
                        dt, (Lp * Dm, Dm), Lp, Bsz, Dm, L, W, stream,
                        dt_bias32=bias if sp else None, dt_softplus=sp)
        outs.append((u, xd, dt))
    torch.cuda.synchronize()
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    want = F.softplus(outs[0][2].double() + bias.double())
    got = outs[1][2].double()
    assert (got > 0).all()
    err = ((got - want).abs() / want).max().item()
    assert err <= 2.0 ** -8, err


def test_mixer_delta_in_conv_proj_matches_delta_in_scan(monkeypatch):
    """Token-major bf16 mixer: delta activated in conv_proj's epilogue
    (VM_DELTA_IN_CONV_PROJ=1) vs inside the scan (default), full sequence and two stateful chunks — they differ
    only by delta's bf16 rounding: 1e-2 relative on outputs, 2e-2 on the fp32 state."""
    from videomamba_amd.mamba_simple import Mamba
    monkeypatch.setenv("VM_MIXER_LAYOUT", "tm")
    torch.manual_seed(6)
    m = Mamba(d_model=128, d_state=16, d_conv=4, expand=2, layer_idx=0).to(DEV, torch.bfloat16)
    x = torch.randn(2, 517, 128, device=DEV).to(torch.bfloat16)
    rel = lambda a, b: ((a.float() - b.float()).norm() / b.float().norm()).item()  # noqa: E731
    res = []
    for pre in ("1", "0"):
        monkeypatch.setenv("VM_DELTA_IN_CONV_PROJ", pre)
        with torch.no_grad():
            full = m(x)
            o1, (c1, s1) = m(x[:, :200], return_state=True)
            o2, (c2, s2) = m(x[:, 200:], state=(c1, s1), return_state=True)
        res.append((full, o1, o2, s2))
    for a, b in zip(res[0], res[1]):
        assert rel(a, b) < 2e-2, rel(a, b)
    assert rel(torch.cat([res[0][1], res[0][2]], 1), res[0][0]) < 1e-2


@pytest.mark.parametrize("n,k,rows,rms,res,epi", [
    (576, 1152, 3144 * 2 + 40, True, True, "1"), (192, 384, 1569, True, True, "1"),
    (192, 384, 700, False, True, "1"), (128, 256, 333, True, False, "0"),
    (64, 64, 130, False, True, "0"), (576, 1152, 257, False, False, "1")])
def test_out_proj_add_norm_matches_library_gemm_and_add_norm(n, k, rows, rms, res, epi,
                                                              monkeypatch):
    """vm_out_proj_add_norm_fwd (out_proj GEMM + residual add + RMSNorm/LayerNorm in one
    launch) against the library GEMM followed by vm_add_norm_fwd: residual_out bit-exact
    and the normalised output within 1 bf16 ulp (in practice identical: same bf16 rounding
    of the hidden, same reduction order).  Ragged row counts (not a multiple of the
    128-row tile), no residual (first block), LayerNorm bias, both epilogue forms."""
    monkeypatch.setenv("VM_OUT_NORM_EPI", epi)
    g = torch.Generator(device=DEV).manual_seed(n + rows)
    y = torch.randn(rows, k, device=DEV, generator=g).to(torch.bfloat16)
    W = (torch.randn(n, k, device=DEV, generator=g) / k ** 0.5).to(torch.bfloat16)
    r = torch.randn(rows, n, device=DEV, generator=g) if res else None
    nw = 1.0 + 0.1 * torch.randn(n, device=DEV, generator=g)
    nb = None if rms else 0.1 * torch.randn(n, device=DEV, generator=g)
    st = torch.cuda.current_stream().cuda_stream
    want = torch.empty(rows, n, device=DEV, dtype=torch.bfloat16)
    want_r = torch.empty(rows, n, device=DEV)
    K.add_norm_raw(F.linear(y, W), r, nw, nb, want, want_r, rows, n, 1e-5, rms, st)
    got = torch.empty_like(want)
    got_r = torch.empty_like(want_r)
    K.out_norm_raw(y, k, W, r, nw, nb, got, got_r, rows, 1e-5, rms, st)
    torch.cuda.synchronize()
    hid = F.linear(y, W).float()
    # the hidden may differ from the library's by a bf16 rounding flip where the fp32
    # accumulation orders differ: residual within one bf16 ulp of the hidden
    tol = (hid.abs() * 2.0 ** -8 + 1e-6)
    assert ((got_r - want_r).abs() <= tol).all()
    _close(got, want, 2e-2)
    # in-place residual (residual_out aliases residual), as the layer loop uses it
    if res:
        r2 = r.clone()
        K.out_norm_raw(y, k, W, r2, nw, nb, got, r2, rows, 1e-5, rms, st)
        torch.cuda.synchronize()
        assert torch.equal(r2, got_r)
