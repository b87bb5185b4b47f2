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
from videomamba_amd import _lib
from videomamba_amd import kernels as K
from videomamba_amd import options

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


@pytest.mark.parametrize("Bz,D,L,N", [(1, 40, 3137, 16),    # several blocks, ragged dim
                                      (64, 72, 300, 16),    # many channels
                                      (2, 24, 777, 8), (3, 20, 100, 4), (1, 8, 0, 16),
                                      (1, 16, 9000, 16)])   # > 8 waves x 512 steps
def test_scan_matches_oracle_random(Bz, D, L, N):
    """Channel-major operands: the time-parallel kernel (its state-split and pipelined
    small-grid forms are picked by grid size: (1, 40, 3137) runs split, (64, 72, 300) the
    one-wave form)."""
    u, delta, A, Bm, Cm, Dv, z, bias, init = _rand_scan(Bz, D, L, N, torch.float32, 11 + L)
    ref_y, ref_h = _oracle_scan(Bz, D, L, N)
    cu = lambda t: None if t is None else t.to(DEV)  # noqa: E731
    y, h = K.selective_scan_fn(cu(u), cu(delta), cu(A), cu(Bm), cu(Cm), cu(Dv), cu(z), cu(bias),
                               True, True, cu(init))
    _close(y, ref_y, 1e-4)
    _close(h, ref_h, 1e-4)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_scan_full_size_chunked_equals_full(dt):
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
def test_scan_token_major_matches_oracle(Bz, D, L, N, segments):
    """Token-major operands take the channel-per-lane kernels: single pass, and the
    segmented summary/carry/final form (options.scan_segments -> the ABI's ``segments``
    argument forces the count; "0" = the cost model's choice)."""
    with options.override(scan_segments=int(segments)):
        _tm_vs_oracle(Bz, D, L, N)


def _tm_vs_oracle(Bz, D, L, N):
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
def test_scan_token_major_full_size_chunked_equals_full(dt, segments):
    """North-star size (D_inner=1152, L=3137), token-major: split scan with the carried
    fp32 state == full scan; and == the channel-major kernels."""
    with options.override(scan_segments=int(segments)):
        _tm_full_size_chunked(dt)


def _tm_full_size_chunked(dt):
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


@pytest.mark.parametrize("segments", ["1", "5"])
@pytest.mark.parametrize("Bz,D,L", [(2, 128, 777), (3, 200, 64), (1, 1152, 3137), (2, 64, 9)])
def test_scan_token_major_bf16_scalar_bc(Bz, D, L, segments):
    """bf16 token-major scan with B/C as scalar loads, single pass and segmented, vs the
    oracle on the same bf16 inputs (one bf16 rounding of the output) and vs the
    channel-major kernel."""
    with options.override(scan_segments=int(segments)):
        _tm_bf16_scalar_bc(Bz, D, L)


def _tm_bf16_scalar_bc(Bz, D, L):
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
def test_scan_mixer_layout_matches_oracle(Bz, D, L, dt, segments):
    """The token-major mixer's exact operand layout (mamba_simple._forward_padded_tm):
    u / delta / y rows (B*Lp, D) with Lp = round_up(L, 8) and zeroed padding rows, z the
    second half of xz rows (B*Lp, 2D), B and C adjacent columns of one x_dbl row
    (B*Lp, R + 2N) — the one-scalar-load B/C form — and an in-place stateful h.  Covers the
    unclamped main loop, the clamped tail and the padded-row zeroing, vs the oracle."""
    with options.override(scan_segments=int(segments)):
        _mixer_layout_scan(Bz, D, L, dt)


def _mixer_layout_scan(Bz, D, L, dt):
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


def _dtproj_case(Bz, D, L, R, seed, exact):
    """Mixer-layout operands for vm_selective_scan_dtproj_fwd: x_dbl rows [dt_low | B | C],
    z inside xz, padded (Lp) rows zero, a zero-padded (D, 32|64) W_dt.  ``exact``: dt_low
    small integers and W_dt multiples of 1/64, so every dt sum is exact in fp32 whatever
    the accumulation order, and dt_ref = bf16(dt_low @ W_dt^T) is the kernel's own dt."""
    N = 16
    E = R + 2 * N
    Lp = (L + 7) // 8 * 8
    g = torch.Generator().manual_seed(seed)
    bf = torch.bfloat16
    if exact:
        dtl = torch.randint(-2, 3, (Bz, L, R), generator=g).float()
        wdt = torch.randint(-4, 5, (D, R), generator=g).float() / 64
    else:
        dtl = torch.randn(Bz, L, R, generator=g)
        wdt = torch.randn(D, R, generator=g) / R ** 0.5
    dtl, wdt = dtl.to(bf), wdt.to(bf)
    dt_ref = (dtl.double() @ wdt.double().t()).float().to(bf)  # (Bz, L, D)
    u = torch.randn(Bz, L, D, generator=g).to(bf)
    z = torch.randn(Bz, L, D, generator=g).to(bf)
    Bm = torch.randn(Bz, L, N, generator=g).to(bf)
    Cm = torch.randn(Bz, L, N, generator=g).to(bf)
    A = -torch.exp(torch.log(torch.arange(1, N + 1).float()).repeat(D, 1)
                   + 0.1 * torch.randn(D, N, generator=g))
    Dv = torch.randn(D, generator=g)
    bias = 0.5 * torch.randn(D, generator=g) - 2.0
    h0 = torch.randn(Bz, D, N, generator=g)
    XD = torch.zeros(Bz, Lp, E, dtype=bf)
    XD[:, :L, :R], XD[:, :L, R:R + N], XD[:, :L, R + N:] = dtl, Bm, Cm
    U = torch.zeros(Bz, Lp, D, dtype=bf)
    XZ = torch.zeros(Bz, Lp, 2 * D, dtype=bf)
    DT = torch.zeros(Bz, Lp, D, dtype=bf)
    U[:, :L], XZ[:, :L, D:], DT[:, :L] = u, z, dt_ref
    wpad = torch.zeros(D, 32 if R <= 32 else 64, dtype=bf)
    wpad[:, :R] = wdt
    dev = lambda t: t.reshape(Bz * Lp, -1).to(DEV) if t.dim() == 3 else t.to(DEV)  # noqa: E731
    return dict(N=N, E=E, Lp=Lp, U=dev(U), XZ=dev(XZ), XD=dev(XD), DT=dev(DT),
                wpad=wpad.to(DEV), A=A.to(DEV).contiguous(), Dv=Dv.to(DEV),
                bias=bias.to(DEV), h0=h0, cpu=(u, dt_ref, z, Bm, Cm, A, Dv, bias))


def _run_dtproj(c, Bz, D, L, R, dtp, segments=1, one_launch=True):
    """dtp: vm_selective_scan_dtproj_fwd; else the scan reading c["DT"] rows.  ``segments``
    (options.scan_segments): 1 = the single pass, 0 = the cost model, > 1 forced."""
    N, E, Lp = c["N"], c["E"], c["Lp"]
    s_u, s_z, s_bc = (Lp * D, 1, D), (Lp * 2 * D, 1, 2 * D), (Lp * E, 1, E)
    XD, XZ = c["XD"], c["XZ"]
    y = torch.full((Bz * Lp, D), 7.0, dtype=torch.bfloat16, device=DEV)
    h = c["h0"].to(DEV).contiguous()
    hs = (D * N, N)
    stream = torch.cuda.current_stream().cuda_stream
    with options.override(scan_segments=segments, scan_one_launch=one_launch):
        if dtp:
            K.scan_dtproj_raw(c["U"], s_u, XD, (Lp * E, E), R, c["wpad"], c["A"],
                              XD[:, R:R + N], s_bc, XD[:, R + N:], s_bc, c["Dv"], XZ[:, D:],
                              s_z, c["bias"], h, hs, h, hs, y, s_u, Lp, Bz, D, L, N, stream)
        else:
            K.scan_raw(c["U"], s_u, c["DT"], s_u, c["A"], XD[:, R:R + N], s_bc, XD[:, R + N:],
                       s_bc, c["Dv"], XZ[:, D:], s_z, c["bias"], True, h, hs, h, hs, y, s_u, Lp,
                       Bz, D, L, N, K.dtype_code(torch.bfloat16), stream)
    return y.view(Bz, Lp, D), h


@pytest.mark.parametrize("Bz,D,L,R", [(2, 256, 301, 36), (3, 128, 20, 12), (1, 384, 1000, 24),
                                      (2, 1152, 3137, 36), (2, 128, 1, 36), (1, 128, 40, 64)])
def test_scan_dtproj_bitwise_equals_dt_rows_then_scan(Bz, D, L, R):
    """vm_selective_scan_dtproj_fwd (dt_proj on the matrix cores inside the scan) on dt sums
    that are exact in fp32 in any order: bit-identical to the single-pass scan reading
    precomputed dt rows bf16(dt_low @ W_dt^T) — the same per-step arithmetic — including
    the 16-step blocks' main loop (L >= 24), the clamped tail (L = 1, 20, ragged ends),
    in-place fp32 state, zeroed padded rows, and every K-chunk count (R = 12 / 24 / 36 /
    64 -> 1 / 2 / 3 / 4 chunks of 16)."""
    c = _dtproj_case(Bz, D, L, R, 100 + L, exact=True)
    y1, h1 = _run_dtproj(c, Bz, D, L, R, True)
    y0, h0 = _run_dtproj(c, Bz, D, L, R, False)
    assert torch.equal(y1, y0)
    assert torch.equal(h1, h0)
    assert not y1[:, L:].float().abs().any()


@pytest.mark.parametrize("R", [12, 36])
def test_scan_dtproj_never_reads_b_columns_as_dt(R):
    """with dt_rank not a multiple of 16 the last dt_low MFMA block spans x_dbl
    columns >= dt_rank, which hold B.  The reference's dt never reads them; the kernel gives
    those k-lanes an out-of-range (zero) load.  An infinite B value at one step must then
    leave every other state's dt finite: bit-identical (NaN payloads included) to the scan
    reading precomputed dt rows."""
    Bz, D, L = 1, 256, 120
    c = _dtproj_case(Bz, D, L, R, 5 + R, exact=True)
    N, Lp = c["N"], c["Lp"]
    c["XD"].view(Bz, Lp, -1)[0, 50, R] = float("inf")  # B[state 0] of step 50
    y1, h1 = _run_dtproj(c, Bz, D, L, R, True)
    y0, h0 = _run_dtproj(c, Bz, D, L, R, False)
    assert torch.equal(y1.view(torch.int16), y0.view(torch.int16))
    assert torch.equal(h1.view(torch.int32), h0.view(torch.int32))
    assert torch.isfinite(h1[:, :, 1:]).all()  # only state 0 saw the infinite B


@pytest.mark.parametrize("one_launch", [True, False])
@pytest.mark.parametrize("Bz,D,L,R,segments", [(1, 1152, 3137, 36, 0), (2, 1152, 3137, 36, 0),
                                                (1, 384, 1000, 12, 0), (3, 256, 777, 24, 40),
                                                (1, 1152, 100, 36, 3), (2, 768, 1569, 36, 0)])
def test_scan_dtproj_segmented_bitwise_equals_dt_rows_then_segmented_scan(Bz, D, L, R, segments,
                                                                         one_launch):
    """ABI v11: at streaming batches the dt_proj-in-scan entry runs the segmented form, each
    segment (<= 64 steps) computing its dt on the matrix cores in conv_proj's arithmetic.  On
    exact dt sums it is bit-identical to the same segmented scan reading precomputed dt rows
    (y, h_last, zeroed padded rows), one-launch and two-launch, for the cost model's segment
    counts at the M / Ti / S shapes of the B = 1 and 2 chunks and forced counts."""
    assert 0 < K.scan_chunk_steps(Bz, D, L, 16, segments) <= K.SCAN_DTPROJ_MAX_SEGMENT
    c = _dtproj_case(Bz, D, L, R, 300 + L + R, exact=True)
    y1, h1 = _run_dtproj(c, Bz, D, L, R, True, segments, one_launch)
    y0, h0 = _run_dtproj(c, Bz, D, L, R, False, segments, one_launch)
    assert torch.equal(y1, y0)
    assert torch.equal(h1, h0)
    assert not y1[:, L:].float().abs().any()


@pytest.mark.parametrize("R", [12, 36])
def test_scan_dtproj_segmented_never_reads_b_columns_as_dt(R):
    """The segmented form's dt operand zeroes the x_dbl columns >= dt_rank (the B values), as
    conv_proj's zero-padded operand does: an infinite B at one step leaves every other
    state's dt finite, bit-identical to the segmented scan reading precomputed dt rows."""
    Bz, D, L = 1, 256, 300
    c = _dtproj_case(Bz, D, L, R, 9 + R, exact=True)
    N, Lp = c["N"], c["Lp"]
    c["XD"].view(Bz, Lp, -1)[0, 50, R] = float("inf")
    y1, h1 = _run_dtproj(c, Bz, D, L, R, True, 0)
    y0, h0 = _run_dtproj(c, Bz, D, L, R, False, 0)
    assert torch.equal(y1.view(torch.int16), y0.view(torch.int16))
    assert torch.equal(h1.view(torch.int32), h0.view(torch.int32))


def test_scan_dtproj_rejects_segments_past_64_steps():
    """The segmented dt_proj-in-scan form holds a segment's dt in LDS: a segment count that
    gives more than 64 steps per segment is refused (VM_E_INVALID, nothing launched) and the
    mixer keeps conv_proj's dt rows there (Mamba._dtp_ok)."""
    Bz, D, L, R = 1, 256, 2000, 36
    assert K.scan_chunk_steps(Bz, D, L, 16, 10) == 200
    c = _dtproj_case(Bz, D, L, R, 11, exact=True)
    with pytest.raises(RuntimeError, match="64 steps"):
        _run_dtproj(c, Bz, D, L, R, True, 10)


@pytest.mark.parametrize("bsz,d_model", [(1, 576), (2, 576), (4, 576), (1, 192), (3, 384)])
def test_mixer_segmented_dtproj_bitwise_equals_conv_proj_dt_rows(bsz, d_model):
    """The streaming-batch mixer with dt_proj inside the segmented scan (round 4; the
    default where its grid fits the chip, forced here by "on") against conv_proj writing
    the dt rows the scan reads (options.scan_dt_proj = "off"):
    bit-identical outputs and states on real-valued weights and inputs — the dt arithmetic
    is conv_proj's own, so moving it changes no result (and chunked == full keeps holding
    whichever form a chunk length picks)."""
    from videomamba_amd.mamba_simple import Mamba
    torch.manual_seed(bsz + d_model)
    m = Mamba(d_model=d_model, layer_idx=0).to(DEV, torch.bfloat16).eval()
    L = 3137
    x = torch.randn(bsz, L, d_model, device=DEV).to(torch.bfloat16)
    hn = torch.empty(1, 1, d_model, device=DEV, dtype=torch.bfloat16).expand(bsz, 3144, d_model)
    pays = K.scan_dtproj_segmented_pays(bsz, m.d_inner, L, 16, DEV)
    assert m._dtp_ok(hn, L) == pays
    with options.override(scan_dt_proj="off"):
        assert not m._dtp_ok(hn, L)
    with options.override(scan_dt_proj="on"):  # any grid
        assert m._dtp_ok(hn, L) == (0 < K.scan_chunk_steps(bsz, m.d_inner, L, 16) <= 64)
    outs = {}
    st0 = m.allocate_state(bsz, dtype=torch.float32)
    st0[1].normal_()
    st0[0].normal_()
    for mode in ("on", "off"):
        st = tuple(s.clone() for s in st0)  # the same entry states for both forms
        with torch.no_grad(), options.override(scan_dt_proj=mode):
            y, (cs, ss) = m(x, state=st, return_state=True)
        outs[mode] = (y, cs, ss)
    for a, b in zip(outs["on"], outs["off"]):
        assert torch.equal(a, b)


@pytest.mark.parametrize("Bz,D,L,R", [(2, 256, 301, 36), (1, 1152, 777, 36)])
def test_scan_dtproj_matches_oracle(Bz, D, L, R):
    """Real-valued dt_low / W_dt: the fused dt_proj + scan against the oracle's scan of
    dt = bf16(dt_low @ W_dt^T) (mamba_simple.py:409-435).  bf16 output 2e-2 abs+rel (an
    fp32 accumulation-order difference can flip a dt rounding); state 1e-3."""
    c = _dtproj_case(Bz, D, L, R, 7 + L, exact=False)
    y, h = _run_dtproj(c, Bz, D, L, R, True)
    u, dt_ref, z, Bm, Cm, A, Dv, bias = c["cpu"]
    tr = lambda t: t.transpose(1, 2).float()  # noqa: E731
    ref_y, ref_h = orc.selective_scan(tr(u), tr(dt_ref), A, tr(Bm), tr(Cm), Dv, tr(z), bias,
                                      True, c["h0"], True)
    _close(y[:, :L].transpose(1, 2), ref_y, 2e-2)
    _close(h, ref_h, 1e-3)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("Bz,D,L,segments", [(1, 1152, 3137, 0), (2, 1152, 3137, 0),
                                              (1, 40, 3137, 0), (3, 64, 1000, 24),
                                              (1, 192, 12545, 0)])
def test_scan_one_launch_matches_two_launch_bitwise(Bz, D, L, segments, dt):
    """The segmented token-major scan as ONE launch (blocks publish their aggregates as
    epoch-tagged granules in a zero-initialised sync buffer and poll the earlier blocks'
    granules) against the two-launch form: bit-identical y and h_last, over repeated
    launches on the same sync buffer (each leaves it valid for the next: epoch = launches
    so far, start count 0, no error)."""
    N, R = 16, 8
    E = R + 2 * N
    Lp = (L + 7) // 8 * 8
    n = Bz * Lp
    u, delta, A, Bm, Cm, Dv, z, bias, init = _rand_scan(Bz, D, L, N, dt, 7 + D + L)
    rows = lambda t: t.transpose(1, 2)  # noqa: E731
    U = torch.zeros(Bz, Lp, D, dtype=dt)
    DL = torch.zeros(Bz, Lp, D, dtype=dt)
    XZ = torch.zeros(Bz, Lp, 2 * D, dtype=dt)
    XD = torch.zeros(Bz, Lp, E, dtype=dt)
    U[:, :L], DL[:, :L], XZ[:, :L, D:] = rows(u), rows(delta), rows(z)
    XD[:, :L, R:R + N], XD[:, :L, R + N:] = rows(Bm), rows(Cm)
    U, DL, XZ, XD = (t.reshape(n, -1).to(DEV) for t in (U, DL, XZ, XD))
    s_u, s_z, s_bc = (Lp * D, 1, D), (Lp * 2 * D, 1, 2 * D), (Lp * E, 1, E)
    A_, Dv_, bias_ = A.to(DEV).contiguous(), Dv.to(DEV), bias.to(DEV)
    sync = torch.zeros(max(K.scan_sync_bytes(Bz, D, L, N, segments), 4), dtype=torch.uint8,
                       device=DEV)
    assert K.scan_sync_bytes(Bz, D, L, N, segments) > 0

    def run(one):
        y = torch.full((n, D), 7.0, dtype=dt, device=DEV)
        h = init.to(DEV).contiguous()
        with options.override(scan_one_launch=one, scan_segments=segments), \
                K.sync_override(sync):
            K.scan_raw(U, s_u, DL, s_u, A_, XD[:, R:R + N], s_bc, XD[:, R + N:], s_bc, Dv_,
                       XZ[:, D:], s_z, bias_, True, h, (D * N, N), h, (D * N, N), y, s_u, Lp,
                       Bz, D, L, N, K.dtype_code(dt), torch.cuda.current_stream().cuda_stream)
        return y, h

    y2, h2 = run(False)
    for k in range(3):
        y1, h1 = run(True)
        torch.cuda.synchronize()
        assert torch.equal(y1, y2) and torch.equal(h1, h2)
        # header after the launch (ABI v9): no timed-out hand-off, the epoch advanced to
        # this launch's tag, the start count back at 0 for the next launch
        head = sync[:16].view(torch.int32).cpu().tolist()
        assert head[0] == 0 and head[1] == k + 1 and head[2] == 0, head
    ref_y, _ = orc.selective_scan(u.float(), delta.float(), A, Bm.float(), Cm.float(), Dv,
                                  z.float(), bias, True, init, True)
    _close(y1.view(Bz, Lp, D)[:, :L].transpose(1, 2), ref_y, 1e-4 if dt == torch.float32 else 2e-2)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_scan_token_major_softplus_both_branches(dt):
    """The single-pass token-major kernel carries delta in log2 units, log2(1 + 2^x) with
    a pass-through above x = 20*log2(e) (vm_scan_seq.hip, LG).  Per-channel biases over
    [-15, 25] put dt + bias on both sides of that threshold and down to deltas of ~1e-7,
    with h0 and h_last, forced single pass (segments=1), vs the oracle's torch softplus:
    1e-4 (fp32 operands) / 2e-2 (bf16 operands, one output rounding) abs+rel."""
    Bz, D, L, N = 2, 128, 400, 16
    u, delta, A, Bm, Cm, Dv, z, _, init = _rand_scan(Bz, D, L, N, dt, 77)
    g = torch.Generator().manual_seed(78)
    delta = (0.5 * torch.randn(Bz, D, L, generator=g)).to(dt)
    bias = torch.linspace(-15.0, 25.0, D)
    ref_y, ref_h = orc.selective_scan(u.float(), delta.float(), A, Bm.float(), Cm.float(), Dv,
                                      z.float(), bias, True, init, True)
    cu = lambda t: _tm(t.to(DEV))  # noqa: E731
    with options.override(scan_segments=1):
        y, h = K.selective_scan_fn(cu(u), cu(delta), A.to(DEV), cu(Bm), cu(Cm), Dv.to(DEV),
                                   cu(z), bias.to(DEV), True, True, init.to(DEV))
    tol = 1e-4 if dt == torch.float32 else 2e-2
    scale = ref_y.abs().max().item()
    _close(y / scale, ref_y / scale, tol)
    _close(h / ref_h.abs().max(), ref_h / ref_h.abs().max(), 1e-4)


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


@pytest.mark.parametrize("rows,cols", [(3144, 576), (37, 192), (5, 1000), (9, 1024), (3, 8)])
@pytest.mark.parametrize("with_res", [False, True])
def test_add_rms_bf16_fast_path_matches_generic_form(rows, cols, with_res):
    """vm_add_norm_fwd's branch-free bf16 / fp32-residual RMSNorm kernel (add_rms_bf16_kernel:
    the block's add+norm) against the same call routed to the dtype-generic vector kernel
    (residual_out requested in bf16 selects it; everything else identical): the fp32
    residual sums, hence the statistics, are the same, so the bf16 outputs must agree
    bitwise; and against the oracle at the bf16 tolerance."""
    lib = _lib.load()
    g = torch.Generator(device=DEV).manual_seed(rows + cols)
    x = torch.randn(rows, cols, device=DEV, generator=g).to(torch.bfloat16)
    res = torch.randn(rows, cols, device=DEV, generator=g) if with_res else None
    w = torch.randn(cols, device=DEV, generator=g)
    stream = torch.cuda.current_stream().cuda_stream
    outs = {}
    for ro_dt in (torch.float32, torch.bfloat16):
        y = torch.empty(rows, cols, device=DEV, dtype=torch.bfloat16)
        ro = torch.empty(rows, cols, device=DEV, dtype=ro_dt)
        rc = lib.vm_add_norm_fwd(x.data_ptr(), K.dtype_code(x.dtype),
                                 res.data_ptr() if res is not None else None,
                                 K.dtype_code(torch.float32), w.data_ptr(), None, y.data_ptr(),
                                 K.dtype_code(y.dtype), ro.data_ptr(), K.dtype_code(ro_dt),
                                 rows, cols, 1e-5, 1, stream)
        assert rc == 0, lib.vm_last_error()
        outs[ro_dt] = (y, ro)
    torch.cuda.synchronize()
    assert torch.equal(outs[torch.float32][0], outs[torch.bfloat16][0])
    assert torch.equal(outs[torch.float32][1].to(torch.bfloat16), outs[torch.bfloat16][1])
    ry, rr = orc.add_norm(x.cpu(), None if res is None else res.cpu(), w.cpu(), None, 1e-5,
                          True, True, True)
    _close(outs[torch.float32][0], ry, 1e-2)
    _close(outs[torch.float32][1], rr, 1e-6)


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
    # rectangular patches (PatchEmbed(patch_size=(ph, pw)), videomamba.py:340-364)
    (torch.bfloat16, 2, 4, 64, 48, (16, 8), 1, 192),  # MFMA path (pw % 8 == 0)
    (torch.bfloat16, 1, 4, 48, 64, (8, 16), 2, 64),   # MFMA path, tubelet 2
    (torch.float32, 2, 4, 12, 8, (4, 2), 1, 16),      # generic path
    (torch.bfloat16, 1, 2, 24, 24, (6, 4), 1, 40),    # generic path, bf16
])
def test_patch_embed_matches_oracle(dt, Bz, T, H, W, P, kt, C):
    ph, pw = (P, P) if isinstance(P, int) else P
    g = torch.Generator().manual_seed(H + C)
    video = torch.randn(Bz, 3, T, H, W, generator=g).to(dt)
    w = (0.02 * torch.randn(C, 3, kt, ph, pw, generator=g)).to(dt)
    b = torch.randn(C, generator=g).to(dt)
    hw = (H // ph) * (W // pw)
    spos = (0.02 * torch.randn(hw, C, generator=g)).to(dt)
    tpos = (0.02 * torch.randn(T // kt, C, generator=g)).to(dt)
    ref = _patch_oracle(video, w, b, spos, tpos, kt, dt)
    cls = torch.randn(C, generator=g).to(dt)
    cls_pos = (0.02 * torch.randn(C, generator=g)).to(dt)
    out = torch.full((Bz, ref.shape[1] + 3, C), 7.0, dtype=dt, device=DEV)
    # ABI v12: the head rows (CLS + its positional embedding, added in the model dtype as
    # the reference's cls_token + pos_embed[:, :1]) and the padding row in the same launch
    K.patch_embed(video.to(DEV), w.to(DEV), b.to(DEV), spos.to(DEV), tpos.to(DEV), out, 2,
                  out.stride(0), cls=cls.to(DEV), cls_pos=cls_pos.to(DEV), pad_rows=1)
    _close(out[:, 2:2 + ref.shape[1]], ref, 1e-5 if dt == torch.float32 else 2e-2)
    head = (cls + cls_pos).to(DEV)  # torch's own add in dt
    assert torch.equal(out[:, :2], head.expand(Bz, 2, C))
    assert not out[:, -1].float().abs().any()


@pytest.mark.parametrize("T,kt,C", [(32, 1, 576), (16, 2, 192), (32, 1, 192), (16, 1, 384)])
def test_patch_embed_kernels_agree_bitwise(T, kt, C):
    """The library picks the patch-embed kernel by token count: the LDS-staged 128x192
    tiles at >= 32768 tokens, the 64x192 register-fragment tiles below.  Both accumulate
    in the same k order and round at the same points, so a clip embedded inside a large
    batch equals the same clip embedded alone, bit for bit.  The large kernel walks its
    tiles in XCD groups of 8 token tiles x C / 192 channel tiles: C = 192, 384, 576 cover
    one to three channel tiles per group, and every batch here ends in a partial group."""
    g = torch.Generator().manual_seed(7 + C)
    bf = torch.bfloat16
    Bz = -(-32768 // ((T // kt) * 196)) + 1  # enough clips for the wide-tile kernel
    video = torch.randn(Bz, 3, T, 224, 224, generator=g).to(bf).to(DEV)
    w = (0.02 * torch.randn(C, 3, kt, 16, 16, generator=g)).to(bf).to(DEV)
    b = torch.randn(C, generator=g).to(bf).to(DEV)
    spos = (0.02 * torch.randn(196, C, generator=g)).to(bf).to(DEV)
    tpos = (0.02 * torch.randn(T // kt, C, generator=g)).to(bf).to(DEV)
    n = (T // kt) * 196
    cls = torch.randn(C, generator=g).to(bf).to(DEV)
    cls_pos = (0.02 * torch.randn(C, generator=g)).to(bf).to(DEV)
    big = torch.full((Bz, n + 8, C), 7.0, dtype=bf, device=DEV)
    K.patch_embed(video, w, b, spos, tpos, big, 1, big.stride(0), cls=cls, cls_pos=cls_pos,
                  pad_rows=7)
    one = torch.full((1, n + 8, C), 7.0, dtype=bf, device=DEV)
    K.patch_embed(video[Bz - 1:].contiguous(), w, b, spos, tpos, one, 1, one.stride(0),
                  cls=cls, cls_pos=cls_pos, pad_rows=7)
    assert torch.equal(big[Bz - 1:], one)
    assert torch.equal(big[:, 0], (cls + cls_pos).expand(Bz, C))
    assert not big[:, n + 1:].float().abs().any()
    one = one[:, :n + 1]
    ref = _patch_oracle(video[Bz - 1:].cpu(), w.cpu(), b.cpu(), spos.cpu(), tpos.cpu(), kt, bf)
    _close(one[:, 1:], ref, 2e-2)


def test_conv_proj_without_dt_matches_with_dt():
    """vm_conv_proj_fwd with dt == NULL (conv + x_proj only) writes the same u and x_dbl
    bits as the full kernel; the full kernel's dt equals x_dbl[:, :R] @ W_dt^T from the
    library GEMM within one bf16 rounding (fp32 accumulation order differs)."""
    from videomamba_amd.mamba_simple import Mamba
    torch.manual_seed(3)
    m = Mamba(d_model=64, d_state=16, d_conv=4, expand=2, layer_idx=0).to(DEV, torch.bfloat16)
    Dm, E, R, W = m.d_inner, m.dt_rank + 2 * m.d_state, m.dt_rank, m.d_conv
    Bsz, L = 3, 301
    Lp = (L + 7) // 8 * 8
    n = Bsz * Lp
    xz = torch.randn(n, 2 * Dm, device=DEV).to(torch.bfloat16)
    cs = torch.randn(Bsz, Dm, W, device=DEV).to(torch.bfloat16)
    _, _, _, cw, cb = m._fp32_params()
    wx_pad, wdt_pad = m._padded_proj_weights()
    st = torch.cuda.current_stream().cuda_stream
    res = []
    for with_dt in (True, False):
        u = torch.empty(n, Dm, device=DEV, dtype=torch.bfloat16)
        xd = torch.empty(n, E, device=DEV, dtype=torch.bfloat16)
        dt = torch.empty(n, Dm, device=DEV, dtype=torch.bfloat16) if with_dt else None
        K.conv_proj_raw(xz, (Lp * 2 * Dm, 2 * Dm), cw, cb, cs, (cs.stride(0), cs.stride(1)),
                        None, (0, 0), wx_pad, E, wdt_pad if with_dt else None, R, u,
                        (Lp * Dm, Dm), xd, (Lp * E, E), dt, (Lp * Dm, Dm), Lp, Bsz, Dm, L, W, st)
        res.append((u, xd, dt))
    torch.cuda.synchronize()
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])
    want = F.linear(res[0][1][:, :R].float(), m.dt_proj.weight.float())
    got = res[0][2].float()
    assert ((got - want).abs() <= want.abs() * 2.0 ** -7 + 1e-3).all()


def test_conv_proj_delta_softplus_epilogue():
    """conv_proj's dt epilogue with dt_softplus: delta = softplus(float(bf16(dt)) + bias)
    rounded to bf16, against torch's fp64 softplus applied to the same kernel's plain dt
    output (one bf16 rounding apart: <= 1 ulp = 2^-8 relative).  u and x_dbl unchanged
    (bitwise).  Includes a stateful first chunk."""
    from videomamba_amd.mamba_simple import Mamba
    torch.manual_seed(5)
    m = Mamba(d_model=96, d_state=16, d_conv=4, expand=2, layer_idx=0).to(DEV, torch.bfloat16)
    Dm, E, R, W = m.d_inner, m.dt_rank + 2 * m.d_state, m.dt_rank, m.d_conv
    Bsz, L = 9, 301  # batch > 8: the softplus epilogue lives in the wide (non-split-K) kernel
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


def test_conv_proj_split_k_conv_state_out():
    """The split-K form writes the new conv state from its staged tile rows (and the old
    state's taps for sequences shorter than the kernel): the last d_conv raw inputs of
    [conv_state | x] per channel (mamba_simple.py:383-399), bit-equal to the wide kernel's
    separate launch, for long and shorter-than-width sequences and several batch rows."""
    from videomamba_amd.mamba_simple import Mamba
    torch.manual_seed(5)
    m = Mamba(d_model=576, d_state=16, d_conv=4, expand=2, layer_idx=0).to(DEV, torch.bfloat16)
    Dm, E, R, W = m.d_inner, m.dt_rank + 2 * m.d_state, m.dt_rank, m.d_conv
    _, _, _, cw, cb = m._fp32_params()
    wx_pad, wdt_pad = m._padded_proj_weights()
    st = torch.cuda.current_stream().cuda_stream
    for L in (2, 61, 777):
        Lp = (L + 7) // 8 * 8
        xz9 = torch.randn(9, Lp, 2 * Dm, device=DEV).to(torch.bfloat16)
        xz9[:, L:] = 0
        cs9 = torch.randn(9, Dm, W, device=DEV).to(torch.bfloat16)
        got = []
        for bsz in (9, 3):  # wide kernel, split-K form
            n = bsz * Lp
            xz = xz9[:bsz].reshape(n, 2 * Dm).contiguous()
            cs = cs9[:bsz].contiguous()
            cso = torch.full((bsz, Dm, W), float("nan"), device=DEV, dtype=torch.bfloat16)
            u = torch.empty(n, Dm, device=DEV, dtype=torch.bfloat16)
            xd = torch.empty(n, E, device=DEV, dtype=torch.bfloat16)
            dt = torch.empty(n, Dm, device=DEV, dtype=torch.bfloat16)
            K.conv_proj_raw(xz, (Lp * 2 * Dm, 2 * Dm), cw, cb, cs, (Dm * W, W), cso,
                            (Dm * W, W), wx_pad, E, wdt_pad, R, u, (Lp * Dm, Dm), xd,
                            (Lp * E, E), dt, (Lp * Dm, Dm), Lp, bsz, Dm, L, W, st)
            got.append(cso[:3])
        torch.cuda.synchronize()
        want = torch.cat([cs9[:3], xz9[:3, :L, :Dm].transpose(1, 2)], dim=-1)[..., -W:]
        assert torch.equal(got[0], want), L
        assert torch.equal(got[1], want), L


@pytest.mark.parametrize("width", [2, 3, 4])
@pytest.mark.parametrize("state_dtype", [torch.float32, torch.bfloat16, None])
def test_conv_proj_wide_kernel_widths_states_short_sequences(width, state_dtype):
    """The wide conv_proj kernel (batch > 8; unconditional buffer loads of clamped window
    rows zeroed by mask, conv-state taps OR-ed in from range-checked loads, u rows as
    range-checked buffer stores) against the oracle's causal conv for every batch row:
    conv widths 2-4 (state taps that do not exist for a narrow kernel), fp32 / bf16 / no
    conv state, sequences shorter than the kernel, shorter than a workgroup's 64 rows (one
    workgroup spans many sequences) and not aligned to it; x_dbl within one bf16 rounding
    of the fp32 projection of the kernel's own u; padding rows zero."""
    from videomamba_amd.mamba_simple import Mamba
    torch.manual_seed(width * 7 + (0 if state_dtype is None else state_dtype.itemsize))
    m = Mamba(d_model=96, d_state=16, d_conv=width, expand=2, layer_idx=0).to(DEV, torch.bfloat16)
    Dm, E, R, W = m.d_inner, m.dt_rank + 2 * m.d_state, m.dt_rank, m.d_conv
    _, _, _, cw, cb = m._fp32_params()
    wx_pad, _ = m._padded_proj_weights()
    st = torch.cuda.current_stream().cuda_stream
    bsz = 11
    for L in (2, 3, 37, 101):
        Lp = (L + 7) // 8 * 8
        n = bsz * Lp
        xz3 = torch.randn(bsz, Lp, 2 * Dm, device=DEV).to(torch.bfloat16)
        xz3[:, L:] = 0
        xz = xz3.reshape(n, 2 * Dm)
        cs = None if state_dtype is None else torch.randn(bsz, Dm, W, device=DEV).to(state_dtype)
        u = torch.full((n, Dm), float("nan"), device=DEV, dtype=torch.bfloat16)
        xd = torch.full((n, E), float("nan"), device=DEV, dtype=torch.bfloat16)
        K.conv_proj_raw(xz, (Lp * 2 * Dm, 2 * Dm), cw, cb, cs,
                        (Dm * W, W) if cs is not None else (0, 0), None, (0, 0), wx_pad, E,
                        None, R, u, (Lp * Dm, Dm), xd, (Lp * E, E), None, None, Lp, bsz, Dm,
                        L, W, st)
        torch.cuda.synchronize()
        u3 = u.view(bsz, Lp, Dm)
        assert not u3[:, L:].float().abs().any(), L  # padding rows: zeros, written
        ref_u, _ = orc.causal_conv1d(xz3[:, :L, :Dm].transpose(1, 2).cpu(), cw.cpu(), cb.cpu(),
                                     True, None if cs is None else cs.cpu())
        got = u3[:, :L].transpose(1, 2).float().cpu()
        tol = ref_u.abs() * 2.0 ** -7 + 1e-5  # one bf16 rounding of the fp32 conv
        assert ((got - ref_u).abs() <= tol).all(), (L, (got - ref_u).abs().max())
        want_xd = F.linear(u.float(), m.x_proj.weight.float())
        assert ((xd.float() - want_xd).abs() <= want_xd.abs() * 2.0 ** -7 + 1e-3).all(), L


@pytest.mark.parametrize("d_model", [576, 96])
def test_conv_proj_split_k_matches_wide_kernel(d_model):
    """vm_conv_proj_fwd runs the split-K form (fixed 128-channel splits of the x_proj
    reduction, vm_conv_proj_sk.hip) for batch <= 8 and the one-workgroup-per-64-rows kernel
    above.  The same clip through both: u bit-identical (same conv arithmetic), x_dbl and dt
    within one bf16 rounding of each other (the fp32 reduction orders differ), both vs the
    oracle's conv and the fp32 projections of the kernel's own u.  d_model 96 -> D = 192
    covers a half-width last split (64 channels)."""
    from videomamba_amd.mamba_simple import Mamba
    torch.manual_seed(d_model)
    m = Mamba(d_model=d_model, d_state=16, d_conv=4, expand=2, layer_idx=0).to(DEV, torch.bfloat16)
    Dm, E, R, W = m.d_inner, m.dt_rank + 2 * m.d_state, m.dt_rank, m.d_conv
    _, _, _, cw, cb = m._fp32_params()
    wx_pad, wdt_pad = m._padded_proj_weights()
    st = torch.cuda.current_stream().cuda_stream
    L = 777
    Lp = (L + 7) // 8 * 8
    outs = []
    xz9 = torch.randn(9, Lp, 2 * Dm, device=DEV).to(torch.bfloat16)
    xz9[:, L:] = 0
    cs9 = torch.randn(9, Dm, W, device=DEV).to(torch.bfloat16)
    for bsz in (9, 1):
        n = bsz * Lp
        xz = xz9[:bsz].reshape(n, 2 * Dm).contiguous()
        cs = cs9[:bsz].contiguous()
        u = torch.empty(n, Dm, device=DEV, dtype=torch.bfloat16)
        xd = torch.empty(n, E, device=DEV, dtype=torch.bfloat16)
        dt = torch.empty(n, Dm, device=DEV, dtype=torch.bfloat16)
        K.conv_proj_raw(xz, (Lp * 2 * Dm, 2 * Dm), cw, cb, cs, (Dm * W, W), None, (0, 0),
                        wx_pad, E, wdt_pad, R, u, (Lp * Dm, Dm), xd, (Lp * E, E), dt,
                        (Lp * Dm, Dm), Lp, bsz, Dm, L, W, st)
        outs.append((u[:Lp], xd[:Lp], dt[:Lp]))
    torch.cuda.synchronize()
    (u9, xd9, dt9), (u1, xd1, dt1) = outs
    assert torch.equal(u9, u1)
    assert not u1[L:].float().abs().any() and not dt1[L:].float().abs().any()
    ulp = lambda t: t.float().abs() * 2.0 ** -7 + 1e-6  # noqa: E731
    assert ((xd9.float() - xd1.float()).abs() <= ulp(xd1)).all()
    want_xd = F.linear(u1.float(), m.x_proj.weight.float())
    assert ((xd1.float() - want_xd).abs() <= want_xd.abs() * 2.0 ** -7 + 1e-3).all()
    want_dt = F.linear(xd1[:, :R].float(), m.dt_proj.weight.float())
    assert ((dt1.float() - want_dt).abs() <= want_dt.abs() * 2.0 ** -7 + 1e-3).all()
    ref_u, _ = orc.causal_conv1d(xz9[:1, :L, :Dm].transpose(1, 2).cpu(), cw.cpu(), cb.cpu(), True,
                                 cs9[:1].cpu())
    _close(u1[:L].t().unsqueeze(0), ref_u, 1e-2)


@pytest.mark.parametrize("d_model", [576, 96])
def test_conv_proj_fused_small_batch_matches_split_k_bitwise(d_model):
    """Small batches run conv + x_proj + dt_proj as one fused launch when out_len >= 24
    (conv_proj_fused_kernel) and as the two split-K launches below that; both sum the same
    fixed 128-channel x_proj partials in split order, so the same clips laid out with
    out_len 16 (split-K) and 32 (fused) must give bit-identical u / x_dbl / dt and new conv
    state — which keeps chunked == full bitwise whatever the chunk length.  Sequence starts
    mid-tile, a carried conv state, 3 batch rows; d_model 96 -> a half-width last split."""
    from videomamba_amd.mamba_simple import Mamba
    torch.manual_seed(d_model + 1)
    m = Mamba(d_model=d_model, d_state=16, d_conv=4, expand=2, layer_idx=0).to(DEV, torch.bfloat16)
    Dm, E, R, W = m.d_inner, m.dt_rank + 2 * m.d_state, m.dt_rank, m.d_conv
    _, _, _, cw, cb = m._fp32_params()
    wx_pad, wdt_pad = m._padded_proj_weights()
    st = torch.cuda.current_stream().cuda_stream
    bsz = 3
    for L in (2, 13, 16):
        x3 = torch.randn(bsz, L, Dm, device=DEV).to(torch.bfloat16)
        z3 = torch.randn(bsz, L, Dm, device=DEV).to(torch.bfloat16)
        cs = torch.randn(bsz, Dm, W, device=DEV).to(torch.bfloat16)
        res = []
        for Lp in (16, 32):  # split-K form, fused form
            n = bsz * Lp
            xz = torch.zeros(bsz, Lp, 2 * Dm, device=DEV, dtype=torch.bfloat16)
            xz[:, :L, :Dm] = x3
            xz[:, :L, Dm:] = z3
            xz = xz.reshape(n, 2 * Dm)
            cso = torch.full((bsz, Dm, W), float("nan"), device=DEV, dtype=torch.bfloat16)
            u = torch.empty(n, Dm, device=DEV, dtype=torch.bfloat16)
            xd = torch.empty(n, E, device=DEV, dtype=torch.bfloat16)
            dt = torch.empty(n, Dm, device=DEV, dtype=torch.bfloat16)
            K.conv_proj_raw(xz, (Lp * 2 * Dm, 2 * Dm), cw, cb, cs, (Dm * W, W), cso,
                            (Dm * W, W), wx_pad, E, wdt_pad, R, u, (Lp * Dm, Dm), xd,
                            (Lp * E, E), dt, (Lp * Dm, Dm), Lp, bsz, Dm, L, W, st)
            res.append((u.view(bsz, Lp, Dm)[:, :L], xd.view(bsz, Lp, E)[:, :L],
                        dt.view(bsz, Lp, Dm)[:, :L], cso))
        torch.cuda.synchronize()
        for a, b in zip(*res):
            assert torch.equal(a, b), L


@pytest.mark.parametrize("m,n,k", [(3144, 2304, 576), (3144, 576, 1152), (1, 576, 1152),
                                   (77, 2304, 576), (600, 64, 192), (5000, 136, 384)])
def test_small_m_linear_matches_fp32_reference(m, n, k):
    """vm_linear_fwd (the B = 1 in_proj / out_proj GEMM) against an fp32 torch reference of
    the same bf16 operands: within one bf16 rounding of the output (fp32 accumulation in
    another order).  Rows are independent of m (bit-equal on a prefix: the chunk-invariance
    property), and a column-sliced output view gets the same bits."""
    torch.manual_seed(m + n + k)
    x = torch.randn(m, k, device=DEV).to(torch.bfloat16)
    w = (torch.randn(n, k, device=DEV) * k ** -0.5).to(torch.bfloat16)
    y = K.linear(x, w)
    ref = x.float() @ w.float().t()
    assert ((y.float() - ref).abs() <= ref.abs() * 2.0 ** -8 + 1e-3).all()
    p = min(m, 37)
    assert torch.equal(K.linear(x[:p].contiguous(), w), y[:p])
    out = torch.full((m, 2 * n), 7.0, device=DEV, dtype=torch.bfloat16)
    K.linear(x, w, out=out[:, n:])
    assert torch.equal(out[:, n:], y) and (out[:, :n] == 7.0).all()


def test_b1_mixer_projections_run_on_the_hip_gemm():
    """The mixer's projections take vm_linear_fwd (the native path) at every batch by
    default (options.projection_gemm = "hip": rows independent of the row count); at one
    clip's token count the mixer output matches the library-GEMM path ("library" mode, the
    round-3 rule) within bf16 rounding."""
    from videomamba_amd.mamba_simple import Mamba, _small_gemm_ok
    torch.manual_seed(0)
    m = Mamba(d_model=576, layer_idx=0).to(DEV, torch.bfloat16).eval()
    x = torch.randn(1, 3137, 576, device=DEV).to(torch.bfloat16)
    hp = torch.zeros(1, 3144, 576, device=DEV, dtype=torch.bfloat16)
    assert _small_gemm_ok(hp.view(3144, 576), m.in_proj.weight, None)
    y = torch.zeros(3144, 1152, device=DEV, dtype=torch.bfloat16)
    assert _small_gemm_ok(y, m.out_proj.weight, None)
    big = torch.zeros(448 * 3144, 1152, device=DEV, dtype=torch.bfloat16)
    assert _small_gemm_ok(big, m.out_proj.weight, None)  # past 2 GB: the persistent form
    with options.override(projection_gemm="library"):
        assert not _small_gemm_ok(hp.view(3144, 576), m.in_proj.weight, None)
        assert not _small_gemm_ok(big, m.out_proj.weight, None)
    del big
    with torch.no_grad():
        y_hip = m(x)
        with options.override(projection_gemm="library", small_gemm_rows=0,
                              row_invariant_gemm_clips=0):
            y_lib = m(x)
    rel = ((y_hip.float() - y_lib.float()).norm() / y_lib.float().norm()).item()
    assert rel < 1e-2, rel


@pytest.mark.parametrize("m,n,k", [(3144, 576, 1152), (100, 192, 384), (1, 576, 1152),
                                   (6288, 576, 1152), (37, 384, 768), (12552, 576, 1152)])
def test_linear_add_norm_bitwise_equals_linear_then_add_norm(m, n, k):
    """vm_linear_add_norm_fwd (out_proj with the next block's residual add + RMSNorm run by
    the last column tile of each 16-row granule) == vm_linear_fwd followed by
    vm_add_norm_fwd, bit for bit (h, the updated fp32 residual, the normalised rows); the
    hand-off counters come back zeroed, so a second launch on the same buffer is exact too."""
    torch.manual_seed(m + n)
    x = torch.randn(m, k, device=DEV).to(torch.bfloat16)
    w = (torch.randn(n, k, device=DEV) / k ** 0.5).to(torch.bfloat16)
    res0 = torch.randn(m, n, device=DEV)
    nw = torch.rand(n, device=DEV) + 0.5
    h_ref = K.linear(x, w)
    res_ref = res0.clone()
    hn_ref = torch.empty(m, n, device=DEV, dtype=torch.bfloat16)
    K.add_norm_raw(h_ref, res_ref, nw, None, hn_ref, res_ref, m, n, 1e-5, True,
                   torch.cuda.current_stream().cuda_stream)
    for _ in range(2):
        res = res0.clone()
        hn = torch.empty(m, n, device=DEV, dtype=torch.bfloat16)
        h = K.linear_add_norm(x, w, res, nw, 1e-5, hn)
        torch.cuda.synchronize()
        assert torch.equal(h, h_ref)
        assert torch.equal(res, res_ref)
        assert torch.equal(hn, hn_ref)
    cnt = K.counter_buffer(x.device, torch.cuda.current_stream().cuda_stream, 0)
    assert not cnt.any()


@pytest.mark.parametrize("m,n,k", [(3144, 576, 1152), (1576, 192, 384), (777, 576, 1152)])
def test_linear_add_norm_one_launch_is_repeatable(m, n, k):
    """The one-launch form of vm_linear_add_norm_fwd (grid <= CUs: the B = 1 out_proj shapes
    of M and Ti): every workgroup runs a share of the next block's add + RMSNorm after its
    tile, waiting on per-row-tile counters (sc1 hand-off).  40 launches on one counter buffer
    are bit-identical to out_proj + vm_add_norm_fwd, finite, and leave the buffer zeroed."""
    torch.manual_seed(m + 7)
    x = torch.randn(m, k, device=DEV).to(torch.bfloat16)
    w = (torch.randn(n, k, device=DEV) / k ** 0.5).to(torch.bfloat16)
    res0 = torch.randn(m, n, device=DEV)
    nw = torch.rand(n, device=DEV) + 0.5
    h_ref = K.linear(x, w)
    res_ref = res0.clone()
    hn_ref = torch.empty(m, n, device=DEV, dtype=torch.bfloat16)
    K.add_norm_raw(h_ref, res_ref, nw, None, hn_ref, res_ref, m, n, 1e-5, True,
                   torch.cuda.current_stream().cuda_stream)
    res = torch.empty_like(res0)
    hn = torch.empty(m, n, device=DEV, dtype=torch.bfloat16)
    bad = 0
    for _ in range(40):
        res.copy_(res0)
        h = K.linear_add_norm(x, w, res, nw, 1e-5, hn)
        bad += int(not (torch.equal(h, h_ref) and torch.equal(res, res_ref)
                        and torch.equal(hn, hn_ref)))
    torch.cuda.synchronize()
    assert bad == 0, bad
    cnt = K.counter_buffer(x.device, torch.cuda.current_stream().cuda_stream, 0)
    assert not cnt.any()


@pytest.mark.parametrize("m,n,k,reps", [(40000, 576, 1152, 20), (100001, 192, 384, 5),
                                        (50003, 384, 768, 5), (1408512, 576, 1152, 4)])
def test_persistent_linear_add_norm_bitwise_and_repeatable(m, n, k, reps):
    """vm_linear_add_norm_fwd at chip-filling row counts: the persistent tile GEMM with the
    next block's add + RMSNorm run per 256-row block by the workgroup of its last column tile
    after the other column tiles' producers count in (vm_gemm_tile.hip NORM).  Every launch
    is bit-identical to the persistent out_proj followed by vm_add_norm_fwd (h, the fp32
    residual updated in place, the normalised rows) and leaves the counters zeroed.  Shapes:
    ragged row blocks for VideoMamba-M / Ti / S out_proj, and the bench's B = 448 out_proj
    (1,408,512 rows: x and the residual past 2 GB)."""
    torch.manual_seed(m + n)
    x = torch.randn(m, k, device=DEV).to(torch.bfloat16)
    w = (torch.randn(n, k, device=DEV) / k ** 0.5).to(torch.bfloat16)
    res0 = torch.randn(m, n, device=DEV)
    nw = torch.rand(n, device=DEV) + 0.5
    h_ref = K.linear(x, w)
    res_ref = res0.clone()
    hn_ref = torch.empty(m, n, device=DEV, dtype=torch.bfloat16)
    K.add_norm_raw(h_ref, res_ref, nw, None, hn_ref, res_ref, m, n, 1e-5, True,
                   torch.cuda.current_stream().cuda_stream)
    res = torch.empty_like(res0)
    hn = torch.empty(m, n, device=DEV, dtype=torch.bfloat16)
    h = torch.empty(m, n, device=DEV, dtype=torch.bfloat16)
    bad = 0
    for _ in range(reps):
        res.copy_(res0)
        hn.fill_(0)
        K.linear_add_norm(x, w, res, nw, 1e-5, hn, h=h)
        bad += int(not (torch.equal(h, h_ref) and torch.equal(res, res_ref)
                        and torch.equal(hn, hn_ref)))
    torch.cuda.synchronize()
    assert bad == 0, bad
    assert torch.isfinite(hn[-1].float()).all()
    cnt = K.counter_buffer(x.device, torch.cuda.current_stream().cuda_stream, 0)
    assert not cnt.any()


@pytest.mark.parametrize("m,n,k", [(70001, 2304, 576), (70001, 576, 1152), (4097, 2304, 576),
                                   (300, 576, 1152), (9001, 768, 192), (9001, 192, 384),
                                   (5555, 1536, 384), (5555, 384, 768), (1, 2304, 576)])
def test_persistent_linear_bitwise_equals_dma_tiles(m, n, k):
    """The persistent 256-row tile GEMM (vm_gemm_tile.hip: persistent workgroups, LDS-DMA
    half-tiles, out^T MFMA tiles stored through v_permlane16_swap) against the 128-row LDS-DMA
    tile kernel on the same operands: bit-identical outputs (every element the same MFMA
    chain in K order), within one bf16 rounding of an fp32 torch reference.  Shapes: the
    mixer's in_proj / out_proj of M, Ti and S, ragged m (a partial last 256-row tile, odd
    tile counts per workgroup, a run that ends mid tile pair, m = 1), both tile widths."""
    torch.manual_seed(m + n + k)
    x = torch.randn(m, k, device=DEV).to(torch.bfloat16)
    w = (torch.randn(n, k, device=DEV) * k ** -0.5).to(torch.bfloat16)
    y_dma = K.linear(x, w, form="dma")
    y_tile = torch.full((m + 3, n), 7.0, device=DEV, dtype=torch.bfloat16)
    K.linear(x, w, out=y_tile[:m], form="persistent")
    torch.cuda.synchronize()
    assert torch.equal(y_tile[:m], y_dma)
    assert (y_tile[m:] == 7.0).all()  # nothing past row m
    ref = x.float() @ w.float().t()
    assert ((y_tile[:m].float() - ref).abs() <= ref.abs() * 2.0 ** -8 + 1e-3).all()


@pytest.mark.parametrize("m,n,k", [(20000, 2304, 576), (20000, 576, 1152)])
def test_persistent_linear_rows_independent_of_m_and_output_stride(m, n, k):
    """Chunk invariance of the projections at chip-filling batches: a row's
    bits do not depend on how many rows the call holds (a prefix run on the LDS-DMA form, a
    middle slice on the persistent form) nor on a column-sliced output view (ldo > n), and
    repeated launches are bit-identical."""
    torch.manual_seed(3 * m + n)
    x = torch.randn(m, k, device=DEV).to(torch.bfloat16)
    w = (torch.randn(n, k, device=DEV) * k ** -0.5).to(torch.bfloat16)
    y = K.linear(x, w, form="persistent")
    assert torch.equal(K.linear(x, w, form="persistent"), y)
    assert torch.equal(K.linear(x[:3001].contiguous(), w, form="dma"), y[:3001])
    assert torch.equal(K.linear(x[5000:17777].contiguous(), w, form="persistent"), y[5000:17777])
    out = torch.full((m, 2 * n), 7.0, device=DEV, dtype=torch.bfloat16)
    K.linear(x, w, out=out[:, n:], form="persistent")
    assert torch.equal(out[:, n:], y) and (out[:, :n] == 7.0).all()
    assert torch.equal(K.linear(x, w), y)  # the auto choice at this size: same bits


def test_persistent_linear_rejects_unsupported_shapes():
    """The persistent form needs no bias and n a multiple of 192 or 256; asked for anyway it
    returns VM_E_INVALID (nothing launched), while the auto form falls back to LDS-DMA tiles."""
    x = torch.randn(4096, 576, device=DEV).to(torch.bfloat16)
    w = torch.randn(200, 576, device=DEV).to(torch.bfloat16)
    with pytest.raises(RuntimeError, match="persistent"):
        K.linear(x, w, form="persistent")
    y = K.linear(x, w)
    assert torch.equal(y, K.linear(x, w, form="dma"))


@pytest.mark.parametrize("m,n,k,past", [(470000, 2304, 576, "out"), (940000, 576, 1152, "x")])
def test_persistent_linear_past_2gb_matches_slices_and_fp32(m, n, k, past):
    """The bench's projection extents: at B = 448 xz is 6.5 GB and y 3.2 GB,
    past every 31-bit buffer offset.  Here the output (in_proj shape, 2.17 GB) or x (out_proj
    shape, 2.17 GB) crosses 2 GB.  Row slices straddling the byte-2^31 row, the first rows and
    the last (partial) tile are bit-equal to the LDS-DMA form run on just those rows (rows do
    not depend on the row count) and within one bf16 rounding of an fp32 torch product."""
    g = torch.Generator(device=DEV).manual_seed(m % 1000 + n)
    x = torch.empty(m, k, device=DEV, dtype=torch.bfloat16)
    for r in range(0, m, 100000):  # fill in slabs: no fp32 copy of the whole operand
        x[r:r + 100000] = torch.randn(min(100000, m - r), k, device=DEV, generator=g)
    w = (torch.randn(n, k, device=DEV, generator=g) * k ** -0.5).to(torch.bfloat16)
    row_bytes = (n if past == "out" else k) * 2
    assert m * row_bytes > 2 ** 31
    y = K.linear(x, w)  # the auto choice: the persistent form (the only one past 2 GB)
    assert torch.equal(K.linear(x, w, form="persistent"), y)
    edge = 2 ** 31 // row_bytes
    for lo, hi in [(0, 700), (edge - 300, edge + 300), ((edge // 256) * 256 - 5, (edge // 256) * 256 + 261),
                   (m - 613, m)]:
        ref_rows = K.linear(x[lo:hi].contiguous(), w, form="dma")
        assert torch.equal(y[lo:hi], ref_rows), (lo, hi)
        ref = x[lo:hi].float() @ w.float().t()
        assert ((y[lo:hi].float() - ref).abs() <= ref.abs() * 2.0 ** -8 + 1e-3).all(), (lo, hi)
    assert torch.isfinite(y[::997].float()).all()


def test_persistent_linear_is_repeatable_at_chip_filling_rows():
    """The persistent GEMM at the C4 B=72 projection shapes (226,368 rows: ~3.5 tiles per
    workgroup run) gives the same bits launch after launch.  Its first build counted the
    previous tile's output stores as ops younger than an awaited LDS-DMA half-tile; a store
    that completed before an older load let a wave read a half-tile that had not landed (1
    launch in 30 differed, scripts/diag/determinism_b72.py)."""
    g = torch.Generator(device=DEV).manual_seed(7)
    m = 72 * 3144
    for n, k in [(2304, 576), (576, 1152)]:
        x = torch.randn(m, k, device=DEV, generator=g).to(torch.bfloat16)
        w = (torch.randn(n, k, device=DEV, generator=g) * k ** -0.5).to(torch.bfloat16)
        r0 = K.linear(x, w, form="persistent")
        bad = sum(int(not torch.equal(K.linear(x, w, form="persistent"), r0)) for _ in range(40))
        assert bad == 0, (n, k, bad)
        del x, w, r0


@pytest.mark.parametrize("d_model", [192, 384, 576])
@pytest.mark.parametrize("bsz", [1, 2, 3, 8])
def test_in_proj_conv_proj_bitwise_equals_in_proj_then_conv_proj(d_model, bsz):
    """vm_in_proj_conv_proj_fwd (in_proj with the conv + SiLU and the x_proj split partials
    in its epilogue, vm_inproj_conv.hip) against the two steps it replaces: vm_linear_fwd
    (in_proj, mamba_simple.py:333-339) then vm_conv_proj_fwd (conv + x_proj + dt_proj,
    :381-416).  z, u, x_dbl, dt and the new conv state are bit-identical — for sequences
    shorter than a 112-row tile and longer than many, chunks padded past their length,
    sequence starts mid-tile (bsz > 1; batch 8, the kernel's maximum), a carried conv state in bf16 / fp32 or none, dt rows
    or none (the scan computes them), and the M-16f chunk shape (3137 tokens)."""
    from videomamba_amd.mamba_simple import Mamba
    torch.manual_seed(d_model + bsz)
    m = Mamba(d_model=d_model, d_state=16, d_conv=4, expand=2, layer_idx=0).to(DEV, torch.bfloat16)
    C, Dm, E, R, W = d_model, m.d_inner, m.dt_rank + 2 * m.d_state, m.dt_rank, m.d_conv
    _, _, _, cw, cb = m._fp32_params()
    wx_pad, wdt_pad = m._padded_proj_weights()
    w_in = m.in_proj.weight
    st = torch.cuda.current_stream().cuda_stream
    cases = [(57, 64, "bf16", True), (100, 112, None, False), (3, 56, "fp32", True),
             (230, 232, "bf16", False)]
    if d_model == 576 and bsz == 1:
        cases.append((3137, 3144, "bf16", False))  # the B = 1 chunk (dt inside the scan)
    for L, Lp, cs_kind, with_dt in cases:
        n = bsz * Lp
        hn = torch.zeros(bsz, Lp, C, device=DEV, dtype=torch.bfloat16)
        hn[:, :L] = torch.randn(bsz, L, C, device=DEV).to(torch.bfloat16)
        hn = hn.view(n, C)
        cs = None
        if cs_kind:
            cs = torch.randn(bsz, Dm, W, device=DEV).to(
                torch.bfloat16 if cs_kind == "bf16" else torch.float32)
        csi_s = (cs.stride(0), cs.stride(1)) if cs is not None else (0, 0)
        outs = []
        for fused in (False, True):
            cso = torch.full((bsz, Dm, W), float("nan"), device=DEV, dtype=torch.bfloat16)
            u = torch.full((n, Dm), float("nan"), device=DEV, dtype=torch.bfloat16)
            xd = torch.full((n, E), float("nan"), device=DEV, dtype=torch.bfloat16)
            dt = torch.full((n, Dm), float("nan"), device=DEV, dtype=torch.bfloat16) if with_dt else None
            xz = torch.full((n, 2 * Dm), float("nan"), device=DEV, dtype=torch.bfloat16)
            if fused:
                assert K.in_proj_conv_proj_fits(C, bsz, Lp, Dm, E, wx_pad.shape[0],
                                                wdt_pad.shape[1], W, with_dt)
                K.in_proj_conv_proj_raw(hn, w_in, xz[:, Dm:], cw, cb, cs, csi_s, cso,
                                        (Dm * W, W), wx_pad, E, wdt_pad, R, u, xd, dt, Lp,
                                        bsz, Dm, L, W, st)
            else:
                K.linear(hn, w_in, out=xz)
                K.conv_proj_raw(xz, (Lp * 2 * Dm, 2 * Dm), cw, cb, cs, csi_s, cso, (Dm * W, W),
                                wx_pad, E, wdt_pad if with_dt else None, R, u, (Lp * Dm, Dm),
                                xd, (Lp * E, E), dt, (Lp * Dm, Dm), Lp, bsz, Dm, L, W, st)
            outs.append((xz[:, Dm:], u, xd, dt, cso))
        torch.cuda.synchronize()
        for name, a, b in zip(("z", "u", "x_dbl", "dt", "conv_state"), *outs):
            if a is None:
                continue
            assert torch.equal(a, b), (L, Lp, cs_kind, name,
                                       (a.float() - b.float()).abs().nan_to_num(9.0).max().item())


def test_in_proj_conv_proj_rejects_unsupported_shapes():
    """vm_in_proj_conv_proj_fits / _fwd refuse what the kernel does not cover (batch > 8,
    chunks under 56 padded tokens, d_inner % 128, in_proj K outside the GEMM's set) — the
    mixer then runs in_proj + conv_proj."""
    assert K.in_proj_conv_proj_fits(576, 1, 3144, 1152, 68, 80, 64, 4, False)
    assert not K.in_proj_conv_proj_fits(576, 9, 3144, 1152, 68, 80, 64, 4, False)
    assert not K.in_proj_conv_proj_fits(576, 1, 48, 1152, 68, 80, 64, 4, False)
    assert not K.in_proj_conv_proj_fits(576, 1, 3144, 1088, 68, 80, 64, 4, False)
    assert not K.in_proj_conv_proj_fits(640, 1, 3144, 1152, 68, 80, 64, 4, False)

