"""Build a probe variant of libvideomamba_hip.so: copy csrc/ to build/var/<name>/, apply the
variant's text replacements, build to tools/probes/var/<name>/libvideomamba_hip.so.  Product
sources stay untouched; scripts/diag/variant_scan.py loads a variant by path.
    python scripts/diag/build_variant.py bc_fixed
"""
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# name -> [(file, old, new)]
VARIANTS = {
    # scans without the one-step-early gate factor (kSeqGateAhead)
    "sc_nogate": [("vm_scan_seq.hip", "constexpr bool kSeqGateAhead = true;", "constexpr bool kSeqGateAhead = false;")],
    # single-pass scan without the one-step-early delta (kSeqDeltaAhead)
    "sc_noahead": [("vm_scan_seq.hip", "constexpr bool kSeqDeltaAhead = true;", "constexpr bool kSeqDeltaAhead = false;")],
    # small-M GEMM with 32-row tiles where 64-row tiles run (out_proj at B = 1: 495 workgroups)
    "lin32": [("vm_gemm.hip", "  const int bm = big ? 128 : 64;", "  const int bm = big ? 128 : 32;"),
              ("vm_gemm.hip", "    else hipLaunchKernelGGL((linear_kernel<64, NKV>), grid, dim3(256), lds, s, p);    \\",
               "    else hipLaunchKernelGGL((linear_kernel<32, NKV>), grid, dim3(256), lds, s, p);    \\")],
    # scan grids without (sc_xcd: single pass) / with (ch_xcd: chunked) the XCD renumbering
    "sc_xcd": [("vm_scan_seq.hip", "constexpr bool kSeqXcdRemap = true;", "constexpr bool kSeqXcdRemap = false;")],
    "ch_xcd": [("vm_scan_seq.hip", "constexpr bool kChunkXcdRemap = false;", "constexpr bool kChunkXcdRemap = true;")],
    # chunked-scan fixed cost: PASS 1 / PASS 2 without their step loops (results wrong)
    "sc_noloop1": [("vm_scan_seq.hip", "  for (int tg = t_beg; tg < t_end; tg += kPF) {",
                    "  for (int tg = t_beg; PASS == 2 && tg < t_end; tg += kPF) {")],
    "sc_noloop2": [("vm_scan_seq.hip", "  for (int tg = t_beg; tg < t_end; tg += kPF) {",
                    "  for (int tg = t_beg; PASS == 1 && tg < t_end; tg += kPF) {")],
    # small-batch conv_proj: the two-launch split-K form instead of the fused kernel
    "cp_splitk": [("vm_conv_proj.hip", "    if (conv_proj_fused_ok(a)) conv_proj_fused_launch(a, st);",
                   "    if (false) conv_proj_fused_launch(a, st);")],
    # small-M GEMM with 64-row tiles at every shape
    "lin64": [("vm_gemm.hip", "  const bool big = (long long)((m + 127) / 128) * nt >= 384;",
               "  const bool big = false;")],
    # split-K conv_proj single-tile latency: only token tile 0 (9 workgroups) of each kernel
    "cx_onetile": [("vm_conv_proj_sk.hip", "  dim3 g1(tiles, q.nsplit);", "  dim3 g1(1, q.nsplit);"),
                   ("vm_conv_proj_sk.hip", "  const dim3 g2(tiles, cblocks);",
                    "  const dim3 g2(1, cblocks);")],
    # no conv + SiLU math (u tile = raw x); no x_proj MFMA
    "cx_noconv": [("vm_conv_proj_sk.hip", "      const bool live = step < p.seqlen && tok < q.ntok && cact;",
                   "      const bool live = step < p.seqlen && tok < q.ntok && cact;\n      al = bl; ah = bh;")],
    "cx_nomfma": [("vm_conv_proj_sk.hip",
                   "  for (int ks = 0; ks < 4; ++ks) {\n    const bf16x8 av = *reinterpret_cast<const bf16x8*>(\n        &sU[(wave",
                   "  for (int ks = 0; ks < 0; ++ks) {\n    const bf16x8 av = *reinterpret_cast<const bf16x8*>(\n        &sU[(wave")],
    # split-K conv_proj pricing (results wrong): no x_proj partial stores / no u stores /
    # no x tile loads
    "cx_nopart": [("vm_conv_proj_sk.hip", "      if (e < p.e) dst[e] = acc[j][rr];",
                   "      if (e < p.e && acc[j][rr] == 1234.5f) dst[e] = acc[j][rr];")],
    "cx_nou": [("vm_conv_proj_sk.hip", "  if (cact) {\n#pragma unroll\n    for (int i = 0; i < 16; ++i) {\n      const int tok = tok0 + t0 + i;",
                "  if (cact && tok0 < 0) {\n#pragma unroll\n    for (int i = 0; i < 16; ++i) {\n      const int tok = tok0 + t0 + i;")],
    "cx_noload": [("vm_conv_proj_sk.hip", "    if (i < 72 * 16 && tok >= 0 && tok < q.ntok && qd * 8 < nch)",
                   "    if (i < 72 * 16 && tok >= 0 && tok < q.ntok && qd * 8 < nch && tok0 < 0)")],
    # dt_proj-in-scan kernel (scan_seq_dtp_kernel) pricing (results wrong): no dt block
    # (dtp_nodt), no per-quad LDS reads of dt (dtp_noquad)
    "dtp_nodt": [("vm_scan_seq.hip", """    if (j == 12) dt_store();""",
                  """    if (j == 12 && tg < 0) dt_store();""")],
    "dtp_noquad": [("vm_scan_seq.hip", """    if ((j & 3) == 0 && j < 12) dqa[(j >> 2) + 1] = dq_read((j >> 2) + 1);""",
                    """    if ((j & 3) == 0 && j < 12 && tg < 0) dqa[(j >> 2) + 1] = dq_read((j >> 2) + 1);""")],
    # small-M GEMM with an unpadded 64-element LDS row and the 16-byte chunks XOR-swizzled
    # by (row & 7) instead of the 72-element padded pitch
    "lin_swz": [("vm_gemm.hip", "constexpr int kLinPitch = 72;  // bf16 per staged row: 64 + 8 pad (144 B)",
                 "constexpr int kLinPitch = 64;  // bf16 per staged row, 16-B chunks XOR-swizzled"),
                ("vm_gemm.hip", "      *reinterpret_cast<i32x4_t*>(&sA[(pc / KQ) * PITCH + (pc % KQ) * 8]) = a[i];",
                 "      *reinterpret_cast<i32x4_t*>(&sA[(pc / KQ) * PITCH + (((pc % KQ) ^ ((pc / KQ) & 7)) * 8)]) = a[i];"),
                ("vm_gemm.hip", "      *reinterpret_cast<i32x4_t*>(&sB[(pc / KQ) * PITCH + (pc % KQ) * 8]) = b[i];",
                 "      *reinterpret_cast<i32x4_t*>(&sB[(pc / KQ) * PITCH + (((pc % KQ) ^ ((pc / KQ) & 7)) * 8)]) = b[i];"),
                ("vm_gemm.hip", """        af[i] = *reinterpret_cast<const bf16x8_t*>(
            &sA[(wm * WM + i * 16 + (lane & 15)) * PITCH + ks * 32 + (lane >> 4) * 8]);""",
                 """        af[i] = *reinterpret_cast<const bf16x8_t*>(
            &sA[(wm * WM + i * 16 + (lane & 15)) * PITCH + (((ks * 4 + (lane >> 4)) ^ (lane & 7)) * 8)]);"""),
                ("vm_gemm.hip", """        bw[j] = *reinterpret_cast<const bf16x8_t*>(
            &sB[(wn * WN + j * 16 + (lane & 15)) * PITCH + ks * 32 + (lane >> 4) * 8]);""",
                 """        bw[j] = *reinterpret_cast<const bf16x8_t*>(
            &sB[(wn * WN + j * 16 + (lane & 15)) * PITCH + (((ks * 4 + (lane >> 4)) ^ (lane & 7)) * 8)]);""")],
    # timing probe: every step reads the segment's first B/C row (L1/K$-resident), so the
    # chunk kernel's time without the per-step scalar-load latency shows (results wrong)
    "bc_fixed": [("vm_scan_seq.hip",
                  "      bc_load(min(t + 1, tlast), bcw[(j + 1) & 1]);",
                  "      bc_load(t_beg, bcw[(j + 1) & 1]);")],
}


def build(name):
    src = os.path.join(ROOT, "videomamba_amd", "csrc")
    work = os.path.join(ROOT, "build", "var", name, "src", "csrc")  # ../../include resolves
    shutil.rmtree(work, ignore_errors=True)
    shutil.copytree(src, work)
    inc = os.path.join(ROOT, "build", "var", name, "include")
    shutil.rmtree(inc, ignore_errors=True)
    shutil.copytree(os.path.join(ROOT, "include"), inc)
    for fname, old, new in VARIANTS[name]:
        p = os.path.join(work, fname)
        s = open(p).read()
        assert s.count(old) >= 1, (name, fname, old)
        open(p, "w").write(s.replace(old, new))
    out = os.path.join(ROOT, "tools", "probes", "var", name)
    os.makedirs(out, exist_ok=True)
    subprocess.check_call(["make", "-C", work, "-j8", f"OUT={out}/libvideomamba_hip.so",
                           f"BUILD={os.path.join(ROOT, 'build', 'var', name, 'obj')}"])


if __name__ == "__main__":
    for n in sys.argv[1:]:
        build(n)
