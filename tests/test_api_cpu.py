"""CPU tests: public API / streaming contract / builder / loader, mirroring the reference's
CPU tests (tests/test_public_api_contract.py, tests/test_videomamba_regressions.py), plus
the C-ABI library load + export check.  No kernel compute happens here (no GPU)."""

import ctypes
import os
import re
from types import SimpleNamespace
from typing import Any

import pytest
import torch

import video_mamba
import videomamba_amd.videomamba as vm_module
from videomamba_amd import _lib
from videomamba_amd.mamba_simple import Mamba
from videomamba_amd.videomamba import PretrainVideoMamba, create_block, load_state_dict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _small_model(**overrides: Any) -> PretrainVideoMamba:
    kwargs: dict = dict(img_size=8, patch_size=4, depth=2, embed_dim=16, channels=3,
                        ssm_cfg={"use_fast_path": False}, fused_add_norm=False, rms_norm=False,
                        residual_in_fp32=False, kernel_size=1, num_frames=4)
    kwargs.update(overrides)
    return PretrainVideoMamba(**kwargs)


def _cfg(**over):
    base = dict(img_size=8, patch_size=4, depth=2, embed_dim=16, channels=3,
                drop_path_rate=0.0, ssm_cfg={"use_fast_path": False}, norm_epsilon=1e-5,
                fused_add_norm=False, rms_norm=False, residual_in_fp32=False, bimamba=True,
                pool_type="cls+avg", kernel_size=1, num_frames=4, use_checkpoint=False,
                checkpoint_num=0, pretrained=None, ckpt_num_frame=4)
    base.update(over)
    return SimpleNamespace(vision_encoder=SimpleNamespace(**base))


# ------------------------------------------------------------------ public API contract
def test_public_all_matches_reference_surface():
    assert set(video_mamba.__all__) == {
        "DeterminismConfig", "ForwardReturnSemantics", "LayerState", "BiMambaRefinerBlock",
        "PretrainVideoMamba", "STREAMING_CONTRACT_VERSION", "StateShape", "StreamingState",
        "add_determinism_args", "allocate_state", "build_videomamba", "configure_determinism",
        "configure_determinism_from_args", "expected_state_shapes", "forward_return_semantics",
        "model_forward_return_semantics", "validate_state"}
    for name in video_mamba.__all__:
        assert hasattr(video_mamba, name)
    assert video_mamba.build_videomamba is vm_module.build_videomamba
    from video_mamba.mamba_simple import Mamba as M2
    assert M2 is Mamba


def test_streaming_contract_allocate_and_validate_cpu():
    model = _small_model()
    state = video_mamba.allocate_state(model, batch_size=2, dtype=torch.float32)
    video_mamba.validate_state(model, state, batch_size=2)
    shapes = video_mamba.expected_state_shapes(model, batch_size=2)
    assert len(shapes) == model.depth
    assert shapes[0].conv_state == (2, model.layers[0].mixer.d_inner, 4)
    assert shapes[0].ssm_state == (2, model.layers[0].mixer.d_inner, 16)
    st_d = video_mamba.allocate_state(model, batch_size=2, as_dict=True)
    video_mamba.validate_state(model, st_d, batch_size=2)
    assert model.expected_state_shapes(2) == shapes


def test_validate_state_error_messages():
    model = _small_model()
    state = video_mamba.allocate_state(model, batch_size=1)
    with pytest.raises(ValueError, match="State length mismatch"):
        video_mamba.validate_state(model, state[:1], batch_size=1)
    with pytest.raises(ValueError, match="State dict keys mismatch"):
        video_mamba.validate_state(model, {0: state[0]}, batch_size=1)
    with pytest.raises(TypeError, match="list, tuple, or dict"):
        video_mamba.validate_state(model, "nope", batch_size=1)
    with pytest.raises(ValueError, match="conv_state shape mismatch"):
        video_mamba.validate_state(model, state, batch_size=2)
    with pytest.raises(ValueError, match="batch_size must be a positive integer"):
        video_mamba.expected_state_shapes(model, 0)
    with pytest.raises(TypeError, match="2-tuple"):
        video_mamba.validate_state(model, [state[0][0], state[1][0]], batch_size=1)


def test_model_contract_metadata_and_forward_semantics():
    model = _small_model(add_pool_norm=True)
    assert model.streaming_contract_version == video_mamba.STREAMING_CONTRACT_VERSION == "1.0.0"
    sem = model.forward_return_semantics()
    assert sem.without_state == "(x_vis, x_pool)"
    assert sem.with_state == "(x_vis, x_pool, next_state)"
    sem2 = _small_model(add_pool_norm=False).forward_return_semantics()
    assert sem2.without_state == "x_vis"
    assert sem2.with_state == "(x_vis, next_state)"
    assert video_mamba.model_forward_return_semantics(model) == sem


def test_configure_determinism_reseeds_torch_rng():
    video_mamba.configure_determinism(seed=1234, deterministic=True)
    x1 = torch.randn(8)
    video_mamba.configure_determinism(seed=1234, deterministic=True)
    x2 = torch.randn(8)
    torch.testing.assert_close(x1, x2)
    torch.use_deterministic_algorithms(False)


def test_determinism_cli_roundtrip():
    import argparse
    p = video_mamba.add_determinism_args(argparse.ArgumentParser())
    args = p.parse_args(["--seed", "7", "--deterministic", "--cudnn-benchmark", "off"])
    cfg = video_mamba.configure_determinism_from_args(args)
    assert cfg.seed == 7 and cfg.deterministic and not cfg.cudnn_benchmark and not cfg.allow_tf32
    torch.use_deterministic_algorithms(False)


# ------------------------------------------------------------------ builder / loader
def test_bimamba_false_is_rejected():
    with pytest.raises(NotImplementedError, match="bimamba=True"):
        _small_model(bimamba=False)


def test_build_videomamba_namespace_with_pretrained(tmp_path):
    ref = _small_model()
    path = tmp_path / "mini_ckpt.pt"
    torch.save(ref.state_dict(), path)
    model = video_mamba.build_videomamba(_cfg(pretrained=str(path)))
    assert isinstance(model, PretrainVideoMamba)
    for k, v in ref.state_dict().items():
        torch.testing.assert_close(model.state_dict()[k], v)


def test_load_state_dict_rejects_wrapped_checkpoint(tmp_path):
    path = tmp_path / "wrapped.pt"
    torch.save({"model": _small_model().state_dict()}, path)
    with pytest.raises(ValueError, match="plain state_dict checkpoint"):
        video_mamba.build_videomamba(_cfg(pretrained=str(path)))


def test_build_videomamba_requires_channels_attr(tmp_path):
    cfg = _cfg()
    del cfg.vision_encoder.channels
    cfg.vision_encoder.in_chans = 3
    with pytest.raises(AttributeError):
        video_mamba.build_videomamba(cfg)


def test_load_state_dict_uses_weights_only(tmp_path, monkeypatch):
    model = _small_model()
    path = tmp_path / "mini_ckpt.pt"
    torch.save(model.state_dict(), path)
    seen = {}
    orig = vm_module.torch.load

    def wrapped(*a, **kw):
        seen.update(kw)
        return orig(*a, **kw)

    monkeypatch.setattr(vm_module.torch, "load", wrapped)
    load_state_dict(str(path), model, ckpt_num_frame=4, num_frames=4)
    assert seen.get("weights_only") is True


def test_load_state_dict_interpolates_pos_embed_for_non_square_target(tmp_path):
    src = _small_model(img_size=8, patch_size=4)
    dst = _small_model(img_size=(8, 12), patch_size=4)
    path = tmp_path / "src.pt"
    torch.save(src.state_dict(), path)
    load_state_dict(str(path), dst, ckpt_num_frame=4, num_frames=4)
    assert dst.pos_embed.shape == (1, 1 + (8 // 4) * (12 // 4), 16)


def test_load_state_dict_interpolates_temporal_embedding(tmp_path):
    src = _small_model(num_frames=4)
    dst = _small_model(num_frames=8)
    path = tmp_path / "src.pt"
    torch.save(src.state_dict(), path)
    load_state_dict(str(path), dst, ckpt_num_frame=4, num_frames=8)
    assert dst.temporal_pos_embedding.shape == (1, 8, 16)
    with pytest.raises(ValueError, match="ckpt_num_frame must be a positive integer"):
        load_state_dict(str(path), dst, ckpt_num_frame=0, num_frames=8)


def test_no_weight_decay_and_num_layers():
    model = _small_model()
    assert "temporal_pos_embedding" in model.no_weight_decay()
    assert model.get_num_layers() == 2


def test_state_dict_keys_match_reference_layout():
    m = _small_model(fused_add_norm=True, rms_norm=True, residual_in_fp32=True)
    keys = set(m.state_dict())
    expect = {"cls_token", "pos_embed", "temporal_pos_embedding", "patch_embed.proj.weight",
              "patch_embed.proj.bias", "norm.weight", "pool_norm.weight", "pool_norm.bias"}
    for i in range(2):
        for k in ("A_log", "D", "in_proj.weight", "conv1d.weight", "conv1d.bias",
                  "x_proj.weight", "dt_proj.weight", "dt_proj.bias", "out_proj.weight"):
            expect.add(f"layers.{i}.mixer.{k}")
        expect.add(f"layers.{i}.norm.weight")
    assert keys == expect


def test_param_counts_match_survey():
    ti = PretrainVideoMamba(depth=24, embed_dim=192, num_frames=8)
    assert sum(p.numel() for p in ti.parameters()) == 6_228_864


# ------------------------------------------------------------------ device guard
def test_mamba_forward_requires_cuda_tensor_inputs():
    model = Mamba(d_model=8, d_state=4, d_conv=2, expand=2, use_fast_path=False,
                  layer_idx=0).eval()
    with pytest.raises(RuntimeError, match="requires CUDA tensors"):
        model(torch.randn(1, 2, 8))


def test_encoder_forward_requires_cuda_tensor_inputs():
    model = _small_model().eval()
    with pytest.raises(RuntimeError, match="requires CUDA tensors"):
        model(torch.randn(1, 3, 4, 8, 8))


def test_tubelet_validation_happens_before_compute():
    model = _small_model(kernel_size=2, num_frames=8)
    x = torch.randn(1, 3, 5, 8, 8)
    with pytest.raises(ValueError, match="must be divisible by tubelet size"):
        model(x, mask=None, use_image=False)
    with pytest.raises(ValueError, match="must be divisible by tubelet size"):
        model.forward_features(x, mask=None, use_image=False)
    with pytest.raises(ValueError, match="x must have shape"):
        model(torch.randn(3, 4, 8, 8))


def test_block_and_refiner_construct():
    b = create_block(16, ssm_cfg={"use_fast_path": False}, rms_norm=False, fused_add_norm=False,
                     residual_in_fp32=False, layer_idx=0)
    assert b.layer_idx == 0 and b.mixer.bimamba is False
    r = video_mamba.BiMambaRefinerBlock(16, layer_idx=3)
    assert r.block_bwd.layer_idx == 1_000_003
    fs, bs = r.allocate_state(2)
    assert fs[0].shape == (2, 32, 4) and bs[1].shape == (2, 32, 16)


def test_rectangular_patch_size_builds_the_reference_conv():
    # the reference's PatchEmbed takes patch_size as (ph, pw) (videomamba.py:340-364)
    m = video_mamba.PretrainVideoMamba(img_size=16, patch_size=(8, 4), depth=1, embed_dim=16,
                                       num_frames=4)
    pe = m.patch_embed
    assert pe.patch_size == (8, 4) and pe.num_patches == 2 * 4
    assert pe.proj.weight.shape == (16, 3, 1, 8, 4) and pe.proj.stride == (1, 8, 4)
    assert m.pos_embed.shape == (1, 1 + 8, 16)
    assert m._spatial_token_grid(16, 16) == (2, 4)


# ------------------------------------------------------------------ C ABI
def test_library_loads_and_exports_every_header_symbol():
    lib = _lib.load()
    assert lib.vm_abi_version() == _lib.ABI_VERSION
    header = open(os.path.join(ROOT, "include", "videomamba_hip.h")).read()
    declared = set(re.findall(r"^\s*(?:int|long long|const char\*)\s+(vm_\w+)\(", header, re.M))
    assert declared == set(_lib.EXPORTED)
    raw = ctypes.CDLL(_lib.LIB_PATH)
    for name in declared:
        assert getattr(raw, name) is not None


def test_abi_rejects_bad_arguments_without_gpu():
    lib = _lib.load()
    rc = lib.vm_selective_scan_fwd(*([None, 0, 0, 0] * 2), None, *([None, 0, 0, 0] * 2),
                                   None, None, 0, 0, 0, None, 0, None, 0, 0, 0, None, 0, 0, 0,
                                   None, 0, 0, 0, 0, 1, 1, 1, 16, 0, 0, None, 0, None, 0, None)
    assert rc == -1
    assert b"null required pointer" in lib.vm_last_error()
    rc = lib.vm_add_norm_fwd(None, 0, None, 0, None, None, None, 0, None, 0, 1, 8, 1e-5, 1, None)
    assert rc == -1


def test_scan_workspace_query_without_gpu():
    lib = _lib.load()
    # small batch, long sequence: the segmented token-major form wants scratch
    assert lib.vm_selective_scan_workspace_bytes(1, 1152, 3137, 16, 0) > 0
    # a chip-filling batch (>= 1.25 waves per SIMD of 64-channel groups) runs single-pass
    assert lib.vm_selective_scan_workspace_bytes(72, 1152, 3137, 16, 0) == 0
    assert lib.vm_selective_scan_workspace_bytes(1, 1152, 3137, 17, 0) == 0
    # an explicit segment request (the ABI's only configuration argument) is honoured
    one = lib.vm_selective_scan_workspace_bytes(2, 64, 100, 16, 1)
    four = lib.vm_selective_scan_workspace_bytes(2, 64, 100, 16, 4)
    # max of the chunked form (one 8-segment block: 9 x 64 x 17 floats per batch row) and
    # the legacy summary / carry / final form (4 x 64 x 33 floats per batch row)
    chunked = 2 * (9 * 64 * 17) * 4
    legacy = 2 * 4 * 64 * (2 * 16 + 1) * 4
    assert one == 0 and four == max(chunked, legacy)
    # the one-launch form's sync buffer: a 16-byte header (error word, epoch, start count),
    # then a {tag, value} granule per (row, 64-channel group, block, 16 states + delta sum,
    # channel)
    assert lib.vm_selective_scan_sync_bytes(2, 64, 100, 16, 4) == 16 + 2 * 1 * 1 * 17 * 64 * 8
    assert lib.vm_selective_scan_sync_bytes(72, 1152, 3137, 16, 0) == 0
    assert lib.vm_selective_scan_sync_bytes(1, 1152, 3137, 16, 0) > 0


def test_scan_segment_cost_model_choices_without_gpu():
    """The measured segment cost model (vm_scan_seq.hip::choose_segments, fitted to
    profiles/r02_scan_segments_sweep.jsonl) as seen through the sync-buffer query:
    nblk blocks of {tag, value} granules per (row, 64-channel group) at M-16f (D = 1152, 18
    groups).  B = 1:
    S = 112 -> 14 blocks of 8 segments (252 workgroups, one per CU); B = 2 .. 8: S = 56 ->
    7 blocks (the round-1 wave-target rule chose 2-3x slower counts there); B >= 72 (1,280+
    waves): single pass, no segments."""
    lib = _lib.load()
    nblk = lambda B, L: (lib.vm_selective_scan_sync_bytes(B, 1152, L, 16, 0) - 16) // (B * 18 * 17 * 64 * 8)  # noqa: E731
    assert nblk(1, 3137) == 14 and nblk(1, 12545) == 14
    assert nblk(2, 3137) == nblk(4, 3137) == nblk(8, 3137) == 7
    assert lib.vm_selective_scan_sync_bytes(72, 1152, 3137, 16, 0) == 0


def test_library_reads_no_environment():
    """The C library has no configuration channel besides its arguments:
    no getenv in any product source."""
    csrc = os.path.join(ROOT, "videomamba_amd", "csrc")
    for name in os.listdir(csrc):
        if name.endswith((".hip", ".h")):
            assert "getenv" not in open(os.path.join(csrc, name)).read(), name


def test_options_override_and_validation():
    from videomamba_amd import options
    assert options.get().mixer_layout == "auto" and options.get().scan_segments == 0
    with options.override(mixer_layout="tm", scan_segments=8) as o:
        assert options.get() is o and o.scan_segments == 8
    assert options.get().mixer_layout == "auto"
    with pytest.raises(ValueError):
        with options.override(mixer_layout="xx"):
            pass


def test_scan_sync_error_word_is_reported_on_the_host():
    """The one-launch scan's bounded hand-off (vm_scan_seq.hip, PASS 3): a block whose wait
    runs out sets word 0 of the sync buffer (and writes NaN outputs).  The host-side check
    reads that word from a host copy — no GPU involved: a clean header is 0, a set word is
    1, a short buffer is rejected, and check paths raise."""
    from videomamba_amd import kernels as K
    lib = _lib.load()
    nbytes = lib.vm_selective_scan_sync_bytes(1, 1152, 3137, 16, 0)
    buf = torch.zeros(nbytes, dtype=torch.uint8)
    assert K.scan_sync_status(buf) == 0
    buf.view(torch.int32)[0] = 1  # what a timed-out block stores
    assert K.scan_sync_status(buf) == 1
    buf.view(torch.int32)[0] = 0
    buf[4:] = 7  # epoch, start count and granules do not count as errors
    assert K.scan_sync_status(buf) == 0
    assert lib.vm_selective_scan_sync_status(buf.data_ptr(), 8) == -1
    assert b"sync header" in lib.vm_last_error()


@pytest.mark.parametrize("embed_dim,depth", [(192, 24), (384, 24), (576, 32)])
@pytest.mark.parametrize("frames", [8, 16])
def test_graph_workspace_covers_first_and_continuation_chunks(embed_dim, depth, frames):
    """StreamingChunkGraph's scratch must fit both chunk kinds: the first chunk scans
    L = T*196 + 1 tokens, continuation chunks L - 1, and the segment cost model may choose
    more segments (more scratch) for L - 1 (Ti-16f at B = 1 needed 11.35 MB for
    L - 1 against 10.14 MB sized for L).  Ti / S / M at 224 px, B = 1 .. 8."""
    from videomamba_amd import kernels as K
    from videomamba_amd.graphs import chunk_workspace_bytes
    m = PretrainVideoMamba(depth=depth, embed_dim=embed_dim, num_frames=frames)
    mx = next(iter(m._mixers()))
    short_wins = 0
    for B in range(1, 9):
        need, sync_need = chunk_workspace_bytes(m, B, frames, 14, 14)
        for L in (frames * 196 + 1, frames * 196):
            assert need >= K.scan_workspace_bytes(B, mx.d_inner, L, mx.d_state), (B, L)
            assert sync_need >= K.scan_sync_bytes(B, mx.d_inner, L, mx.d_state), (B, L)
        L = frames * 196 + 1
        short_wins += (K.scan_workspace_bytes(B, mx.d_inner, L - 1, mx.d_state)
                       > K.scan_workspace_bytes(B, mx.d_inner, L, mx.d_state))
    if (embed_dim, frames) == (192, 16):
        assert short_wins > 0  # the case the first-chunk-only sizing missed


def test_conv_proj_wide_offset_limit_is_rejected_on_the_host():
    """The wide conv_proj kernel (batch > 8) addresses x rows, the conv state and u rows
    through buffer resources with 31-bit offsets; vm_conv_proj_fwd rejects shapes past them
    before any HIP call (pointers here are never dereferenced): a 300k-token sequence of
    xz at D = 1152 is past the limit."""
    lib = _lib.load()
    D, E, Ep, R = 1152, 68, 80, 36
    fake = lambda i: ctypes.c_void_p((i + 1) << 20)  # noqa: E731  16-byte aligned, unused

    def call(L, batch):
        Lp = L
        return lib.vm_conv_proj_fwd(
            fake(0), Lp * 2 * D, 2 * D, fake(1), fake(2),
            None, 0, 0, 0, None, 0, 0, 0,
            fake(3), E, Ep, None, R, 0,
            fake(4), Lp * D, D, fake(5), Lp * E, E, None, 0, 0,
            None, 0, Lp, batch, D, L, 4, _lib.VM_DTYPE_BF16, None, 0, None)

    assert call(300_000, 9) == -1
    assert b"31-bit" in lib.vm_last_error()
    assert call(300_000, 0) == 0  # empty batch: nothing to launch, nothing to check


def test_conv_proj_fits_query_routes_long_sequences_to_the_unfused_path():
    """the wide conv_proj form's 31-bit offsets reject ~230k-token sequences at
    batch > 8; vm_conv_proj_fits reports that on the host and the mixer's fused-path test
    mirrors it, so such a forward takes the unfused conv + projection path instead of
    raising.  Small batches (split-K / fused forms, 64-bit addressing) always fit."""
    from videomamba_amd import kernels as K
    from videomamba_amd.mamba_simple import Mamba
    D, E = 1152, 68
    fits = lambda B, L: K.conv_proj_fits(B, L, L, D, E, 64, (L * 2 * D, 2 * D), D, None, 4)  # noqa: E731
    assert fits(9, 3144) and fits(448, 3144) and fits(8, 300_000)
    assert not fits(9, 300_000)
    mx = Mamba(d_model=576).to(torch.bfloat16)
    shape_only = lambda B, L: torch.empty(1, 1, 576, dtype=torch.bfloat16).expand(B, L, 576)  # noqa: E731
    assert mx._fused_conv_proj_ok(shape_only(9, 3144), 3137)
    assert not mx._fused_conv_proj_ok(shape_only(9, 300_000), 300_000)
    assert not mx._dtp_ok(shape_only(9, 300_000), 300_000)
    assert mx._fused_conv_proj_ok(shape_only(8, 300_000), 300_000)


def test_linear_rejects_unsupported_k_before_launch():
    """vm_linear_fwd validates k against the unrolled K-step counts it is built
    for and returns VM_E_INVALID (no launch, nothing written) for any other multiple of 64."""
    lib = _lib.load()
    fake = lambda i: ctypes.c_void_p((i + 1) << 20)  # noqa: E731  never dereferenced
    for k in (64, 256, 1024):
        rc = lib.vm_linear_fwd(fake(0), k, fake(1), k, None, fake(2), 64, 128, 64, k,
                               _lib.VM_DTYPE_BF16, None)
        assert rc == -1 and b"k = " in lib.vm_last_error(), k


def test_sync_rearm_clears_only_the_error_word():
    """re-arming a sync buffer after a reported timeout zeroes word 0 (the error
    word) only; the epoch (word 1) keeps growing so stale granules of earlier launches never
    carry a later launch's tag."""
    from videomamba_amd import kernels as K
    buf = torch.zeros(64, dtype=torch.uint8)
    words = buf.view(torch.int32)
    words[0], words[1], words[2] = 1, 41, 3
    with pytest.raises(RuntimeError):
        K._SYNC[("cpu", None, 0)] = buf
        try:
            K.check_scan_sync()
        finally:
            del K._SYNC[("cpu", None, 0)]
    assert words[0] == 0 and words[1] == 41 and words[2] == 3
