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
    # the sources as they stand when built (a same-box baseline for a change under test)
    "base": [],
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
    # one-launch chunked scan pricing (results wrong): the PASS 1 (ch_noloop1) / PASS 2
    # (ch_noloop2) step loop skipped inside the same launch
    "ch_noloop1": [("vm_scan_seq.hip", "    for (int tg = t_beg; tg < t_end; tg += kPF) {",
                    "    for (int tg = t_beg; EMIT && tg < t_end; tg += kPF) {")],
    "ch_noloop2": [("vm_scan_seq.hip", "    for (int tg = t_beg; tg < t_end; tg += kPF) {",
                    "    for (int tg = t_beg; !EMIT && tg < t_end; tg += kPF) {")],
    # dt_proj-in-scan kernel with the inline-asm d16_hi u / z loads and fp32 dt block (the
    # round-5 A/B, measured slower: DESIGN.md §3.1.1; built from LEGACY_REV)
    "dtp_d16": [("vm_scan_seq.hip", "constexpr bool kDtpD16 = false;", "constexpr bool kDtpD16 = true;")],
    # chunked scan: the two waves of each SIMD (w, w + 4) swap the raised issue priority
    # every kPF steps, so neither finishes its step loop far ahead of the other (round 6)
    "ch_prio_toggle": [("vm_scan_seq.hip",
                        "    for (int tg = t_beg; tg < t_end; tg += kPF) {\n#pragma unroll\n      for (int j = 0; j < kPF; ++j) {\n        const int t = tg + j;\n        const bool live = t < t_end;",
                        "    for (int tg = t_beg; tg < t_end; tg += kPF) {\n      if ((((tg - t_beg) / kPF) + (wave >> 2)) & 1) __builtin_amdgcn_s_setprio(1);\n      else __builtin_amdgcn_s_setprio(0);\n#pragma unroll\n      for (int j = 0; j < kPF; ++j) {\n        const int t = tg + j;\n        const bool live = t < t_end;")],
    # the same with a swap every 2 kPF steps
    "ch_prio_toggle2": [("vm_scan_seq.hip",
                        "    for (int tg = t_beg; tg < t_end; tg += kPF) {\n#pragma unroll\n      for (int j = 0; j < kPF; ++j) {\n        const int t = tg + j;\n        const bool live = t < t_end;",
                        "    for (int tg = t_beg; tg < t_end; tg += kPF) {\n      if ((((tg - t_beg) / (2 * kPF)) + (wave >> 2)) & 1) __builtin_amdgcn_s_setprio(1);\n      else __builtin_amdgcn_s_setprio(0);\n#pragma unroll\n      for (int j = 0; j < kPF; ++j) {\n        const int t = tg + j;\n        const bool live = t < t_end;")],
    # the same with one swap, at the middle of the segment
    "ch_prio_half": [("vm_scan_seq.hip",
                        "    for (int tg = t_beg; tg < t_end; tg += kPF) {\n#pragma unroll\n      for (int j = 0; j < kPF; ++j) {\n        const int t = tg + j;\n        const bool live = t < t_end;",
                        "    for (int tg = t_beg; tg < t_end; tg += kPF) {\n      if ((2 * (tg - t_beg) + kPF >= t_end - t_beg) != ((wave >> 2) & 1)) __builtin_amdgcn_s_setprio(1);\n      else __builtin_amdgcn_s_setprio(0);\n#pragma unroll\n      for (int j = 0; j < kPF; ++j) {\n        const int t = tg + j;\n        const bool live = t < t_end;")],
    # bench scan with its LDS dynamic (the compiler's occupancy target ignores it) and a
    # 5-waves-per-SIMD register target (96 VGPRs): at run time LDS still holds it to 4 waves
    # per SIMD, which leaves 128 registers per SIMD for the other sub-batch stream's
    # add + RMSNorm waves (40 each) beside it (round 6)
    "dtp_dyn5": [('vm_scan_seq.hip', '  __shared__ __attribute__((aligned(16))) bf16_t sW[NW][64 * KP];\n  constexpr int DR = kDtRow;\n  __shared__ __attribute__((aligned(16))) uint32_t sD[NW][64 * DR];\n', '  constexpr int DR = kDtRow;\n  extern __shared__ __attribute__((aligned(16))) char dtp_dsm[];\n  auto& sW = *reinterpret_cast<bf16_t (*)[NW][64 * KP]>(dtp_dsm);\n  auto& sD = *reinterpret_cast<uint32_t (*)[NW][64 * DR]>(dtp_dsm + sizeof(bf16_t) * NW * 64 * KP);\n'), ('vm_scan_seq.hip', 'template <int NKS>\n__global__ __launch_bounds__(64 * kSeqNW) void scan_seq_dtp_kernel', 'static size_t dtp_lds(int nks) { return kSeqNW * 64 * ((16 * nks + 4) * 2 + kDtRow * 4); }\n\ntemplate <int NKS>\n__global__ __launch_bounds__(64 * kSeqNW) __attribute__((amdgpu_waves_per_eu(5))) void scan_seq_dtp_kernel'), ('vm_scan_seq.hip', 'hipLaunchKernelGGL(scan_seq_dtp_kernel<1>, grid, dim3(64 * kSeqNW), 0, s, p, q)', 'hipLaunchKernelGGL(scan_seq_dtp_kernel<1>, grid, dim3(64 * kSeqNW), dtp_lds(1), s, p, q)'), ('vm_scan_seq.hip', 'hipLaunchKernelGGL(scan_seq_dtp_kernel<2>, grid, dim3(64 * kSeqNW), 0, s, p, q)', 'hipLaunchKernelGGL(scan_seq_dtp_kernel<2>, grid, dim3(64 * kSeqNW), dtp_lds(2), s, p, q)'), ('vm_scan_seq.hip', 'hipLaunchKernelGGL(scan_seq_dtp_kernel<3>, grid, dim3(64 * kSeqNW), 0, s, p, q)', 'hipLaunchKernelGGL(scan_seq_dtp_kernel<3>, grid, dim3(64 * kSeqNW), dtp_lds(3), s, p, q)'), ('vm_scan_seq.hip', 'hipLaunchKernelGGL(scan_seq_dtp_kernel<4>, grid, dim3(64 * kSeqNW), 0, s, p, q)', 'hipLaunchKernelGGL(scan_seq_dtp_kernel<4>, grid, dim3(64 * kSeqNW), dtp_lds(4), s, p, q)')],
    # VERDICT r5 #2 pricing (results wrong): the persistent in_proj's x-half tiles run a
    # depthwise causal conv (4 taps over tokens: DPP row shifts within each 16-token MFMA
    # block, the previous block's last lanes by row rotation) + SiLU on their bf16 outputs
    # before the store, as a conv fold into the GEMM epilogue would (constant weights, no
    # cross-wave / cross-tile halo, no sequence starts: a lower bound of that epilogue's cost)
    "tg_convpx": [("vm_gemm_tile.hip", "__device__ __forceinline__ int tg_slot(int row, int chunk)",
                   "__device__ __forceinline__ uint32_t tg_conv_silu(uint32_t cur, uint32_t prv, float wb) {\n"
                   "  const uint32_t s1 = __builtin_amdgcn_update_dpp((int)__builtin_amdgcn_mov_dpp((int)prv, 0x121, 0xf, 0xf, false), (int)cur, 0x111, 0xf, 0xf, false);\n"
                   "  const uint32_t s2 = __builtin_amdgcn_update_dpp((int)__builtin_amdgcn_mov_dpp((int)prv, 0x122, 0xf, 0xf, false), (int)cur, 0x112, 0xf, 0xf, false);\n"
                   "  const uint32_t s3 = __builtin_amdgcn_update_dpp((int)__builtin_amdgcn_mov_dpp((int)prv, 0x123, 0xf, 0xf, false), (int)cur, 0x113, 0xf, 0xf, false);\n"
                   "  float r[2];\n"
                   "#pragma unroll\n"
                   "  for (int e = 0; e < 2; ++e) {\n"
                   "    auto f = [&](uint32_t v) { return e ? __uint_as_float(v & 0xffff0000u) : __uint_as_float(v << 16); };\n"
                   "    float c = wb * f(s3);\n"
                   "    c = fmaf(wb + 0.1f, f(s2), c);\n"
                   "    c = fmaf(wb + 0.2f, f(s1), c);\n"
                   "    c = fmaf(wb + 0.3f, f(cur), c);\n"
                   "    r[e] = c * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(c * -1.44269504f));\n"
                   "  }\n"
                   "  return tg_pack(r[0], r[1]);\n"
                   "}\n\n"
                   "__device__ __forceinline__ int tg_slot(int row, int chunk)"),
                  ("vm_gemm_tile.hip",
                   "          const uint32_t a0 = tg_pack(A[0], A[1]), a1 = tg_pack(A[2], A[3]);\n"
                   "          const uint32_t b0 = tg_pack(B[0], B[1]), b1 = tg_pack(B[2], B[3]);\n",
                   "          uint32_t a0 = tg_pack(A[0], A[1]), a1 = tg_pack(A[2], A[3]);\n"
                   "          uint32_t b0 = tg_pack(B[0], B[1]), b1 = tg_pack(B[2], B[3]);\n"
                   "          if (!NORM && col_a < (p.n >> 1)) {\n"
                   "            const tg_f32x4& PA = acc[h][i > 0 ? i - 1 : 0][ia / TNH][ia % TNH];\n"
                   "            const tg_f32x4& PB = acc[h][i > 0 ? i - 1 : 0][ib / TNH][ib % TNH];\n"
                   "            const bool pr = i > 0;\n"
                   "            const uint32_t p0 = pr ? tg_pack(PA[0], PA[1]) : 0u, p1 = pr ? tg_pack(PA[2], PA[3]) : 0u;\n"
                   "            const uint32_t p2 = pr ? tg_pack(PB[0], PB[1]) : 0u, p3 = pr ? tg_pack(PB[2], PB[3]) : 0u;\n"
                   "            const float wb = 0.01f * static_cast<float>(col_a & 15);\n"
                   "            a0 = tg_conv_silu(a0, p0, wb);\n"
                   "            a1 = tg_conv_silu(a1, p1, wb + 0.001f);\n"
                   "            b0 = tg_conv_silu(b0, p2, wb + 0.002f);\n"
                   "            b1 = tg_conv_silu(b1, p3, wb + 0.003f);\n"
                   "          }\n")],
    # B = 1 kernel boundaries: in_proj + conv's u / z / x_proj-partial stores write-through
    # (sc1), so the ~22 MB they leave dirty in L2 drains during the kernel instead of at the
    # boundary (MI355X_MICROARCH.md "boundary": + bytes / 6 TB/s)
    "wt_ic": [("vm_inproj_conv.hip",
               "        *reinterpret_cast<uint4*>(q.z + (long long)gm * q.ldz + (n0 - p.dim) + cq * 8) =\n"
               "            *reinterpret_cast<const uint4*>(&sO[row * kIcPitch + cq * 8]);",
               "        __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<const int __attribute__((ext_vector_type(4)))*>(&sO[row * kIcPitch + cq * 8]),\n"
               "            __builtin_amdgcn_make_buffer_rsrc(q.z, 0, 0x7ffffff0, 0x00020000), static_cast<int>(((long long)gm * q.ldz + (n0 - p.dim) + cq * 8) * 2), 0, 16);"),
              ("vm_inproj_conv.hip",
               "    if (tok < q.ntok) *reinterpret_cast<uint32_t*>(p.u + (long long)tok * p.u_tl + c) = upk[i];",
               "    if (tok < q.ntok) __hip_atomic_store(reinterpret_cast<uint32_t*>(p.u + (long long)tok * p.u_tl + c), upk[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);"),
              ("vm_inproj_conv.hip",
               "        *reinterpret_cast<float4*>(q.part + ((long long)sp * q.ntok + tok) * q.ep + 4 * qd) =\n"
               "            *reinterpret_cast<const float4*>(&sP[r * kPP + 4 * qd]);",
               "        __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<const int __attribute__((ext_vector_type(4)))*>(&sP[r * kPP + 4 * qd]),\n"
               "            __builtin_amdgcn_make_buffer_rsrc(q.part, 0, 0x7ffffff0, 0x00020000), static_cast<int>((((long long)sp * q.ntok + tok) * q.ep + 4 * qd) * 4), 0, 16);")],
    # the same for add + RMSNorm's hn / residual stores, the scans' y stores and the
    # 128-row GEMM's output stores (wt_all = all four kernels of the B = 1 layer)
    "wt_rest": [("vm_norm.hip", "    __builtin_amdgcn_raw_buffer_store_b64(o2, orr, off(j, 2), 0, 0);",
                 "    __builtin_amdgcn_raw_buffer_store_b64(o2, orr, off(j, 2), 0, 16);"),
                ("vm_norm.hip", "      __builtin_amdgcn_raw_buffer_store_b128(r4, ror, off(j, 4), 0, 0);",
                 "      __builtin_amdgcn_raw_buffer_store_b128(r4, ror, off(j, 4), 0, 16);"),
                ("vm_scan_seq.hip", "    __builtin_amdgcn_raw_buffer_store_b16(v, r, voff, soff, 0);",
                 "    __builtin_amdgcn_raw_buffer_store_b16(v, r, voff, soff, 16);"),
                ("vm_gemm.hip", "        *reinterpret_cast<uint4*>(p.out + (long long)gm * p.ldo + gn) = v;",
                 "        typedef __attribute__((__vector_size__(4 * sizeof(int)))) int v4w;\n"
                 "        __builtin_amdgcn_raw_buffer_store_b128(v4w{(int)v.x, (int)v.y, (int)v.z, (int)v.w},\n"
                 "            __builtin_amdgcn_make_buffer_rsrc(p.out, 0, 0x7ffffff0, 0x00020000), static_cast<int>(((long long)gm * p.ldo + gn) * 2), 0, 16);")],
    # x_dbl reduce at B = 1: each block sums the tokens of the row tiles in_proj + conv ran on
    # its own XCD, so the split partials it loads sit in that XCD's L2 (same bits)
    "xr_xcd": [("vm_inproj_conv.hip", "// x_dbl = bf16(sum of the split partials in split order) — xdbl_dt_tm_kernel's sum (from\n// 0, split 0 first, fp32) without its dt phase, one thread per (token, 4 columns) so the\n// whole reduction is one round of loads (that kernel's 64-token tiles take two dependent\n// rounds on a 50-workgroup grid at B = 1).  dt == NULL only (the scan computes dt).\ntemplate <int NSPL>\n__global__ __launch_bounds__(256) void xdbl_reduce_kernel(const InConvParams q) {\n  const ConvProjTmArgs& p = q.a;\n  const int q4 = (p.e + 3) >> 2;\n  const int it = blockIdx.x * 256 + threadIdx.x;\n  if (it >= q.ntok * q4) return;\n  const int t = it / q4, e0 = (it - t * q4) * 4;",
                "// The token range [lo, hi) of the row tiles whose split 0 ran on XCD x in inproj_conv_kernel\n// (its XCD-contiguous numbering of the x tiles: XCD x took logical tiles [start, start + count))\n__device__ __forceinline__ void ic_xcd_tokens(const InConvParams& q, int x, int& lo, int& hi) {\n  const int nwg = q.nxr * q.nsplit, qq = nwg >> 3, rr = nwg & 7;\n  const int start = x < rr ? x * (qq + 1) : rr * (qq + 1) + (x - rr) * qq;\n  const int end = start + qq + (x < rr ? 1 : 0);\n  const int rt_a = (start + q.nsplit - 1) / q.nsplit, rt_b = (end + q.nsplit - 1) / q.nsplit;\n  lo = min(rt_a * kIcOut, q.ntok);\n  hi = min(rt_b * kIcOut, q.ntok);\n}\n\n// x_dbl = bf16(sum of the split partials in split order) — xdbl_dt_tm_kernel's sum (from\n// 0, split 0 first, fp32) without its dt phase, one thread per (token, 4 columns) so the\n// whole reduction is one round of loads (that kernel's 64-token tiles take two dependent\n// rounds on a 50-workgroup grid at B = 1).  dt == NULL only (the scan computes dt).  Block b\n// runs on XCD b % 8 (round-robin dispatch; placement is a speed choice only) and sums the\n// tokens of the row tiles inproj_conv_kernel ran there, so its partial loads hit that XCD's L2.\ntemplate <int NSPL>\n__global__ __launch_bounds__(256) void xdbl_reduce_kernel(const InConvParams q) {\n  const ConvProjTmArgs& p = q.a;\n  const int q4 = (p.e + 3) >> 2;\n  int lo, hi;\n  ic_xcd_tokens(q, blockIdx.x & 7, lo, hi);\n  const int it = lo * q4 + (blockIdx.x >> 3) * 256 + threadIdx.x;\n  if (it >= hi * q4) return;\n  const int t = it / q4, e0 = (it - t * q4) * 4;"),
               ("vm_inproj_conv.hip", '    const unsigned blocks = static_cast<unsigned>((ntok * ((e + 3) / 4) + 255) / 256);',
                "    // 8 x (the most tokens any XCD's row tiles hold) threads, in 256-thread blocks\n    int most = 0;\n    {\n      const int nwg = q.nxr * q.nsplit, qq = nwg >> 3, rr = nwg & 7;\n      for (int x = 0; x < 8; ++x) {\n        const int start = x < rr ? x * (qq + 1) : rr * (qq + 1) + (x - rr) * qq;\n        const int end = start + qq + (x < rr ? 1 : 0);\n        const long long lo = std::min<long long>((start + q.nsplit - 1) / q.nsplit * (long long)kIcOut, ntok);\n        const long long hi = std::min<long long>((end + q.nsplit - 1) / q.nsplit * (long long)kIcOut, ntok);\n        most = std::max(most, static_cast<int>(hi - lo));\n      }\n    }\n    const unsigned blocks = 8u * static_cast<unsigned>((most * ((e + 3) / 4) + 255) / 256);")],
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
    # persistent GEMM: s_setprio around each MFMA quadrant (tg_prio1) / waves 4-7 at
    # priority 1 throughout (tg_prio2)
    # persistent out_proj + add + RMSNorm (vm_gemm_tile.hip NORM) pricing: no norm rows
    # (polls / barriers / hand-off kept; results wrong), 4 rows in flight per wave, h read
    # back without sc1 (timing only)
    "tn_nonorm": [("vm_gemm_tile.hip", "    for (int g = 0; g < RPW; g += kTileNormRows) {",
                   "    for (int g = 0; g < 0; g += kTileNormRows) {")],
    "tn_rows4": [("vm_gemm_tile.hip", "constexpr int kTileNormRows = 8;", "constexpr int kTileNormRows = 4;")],
    "tn_plainh": [("vm_gemm_tile.hip", "          const auto v = __builtin_amdgcn_raw_buffer_load_b64(hr, c2[j] + oh, 0, kTileSC1);",
                   "          const auto v = __builtin_amdgcn_raw_buffer_load_b64(hr, c2[j] + oh, 0, 0);")],
    # persistent GEMM: the tile's stores in two halves (A-top after phase 1, A-bottom after
    # phase 3 of the last K-tile)
    "tg_split": [("vm_gemm_tile.hip", "constexpr bool kTileSplitStore = false;", "constexpr bool kTileSplitStore = true;")],
    # chunked scan: B|C rows one step ahead with a wait every step (the round-4 form)
    "ch_bc1": [("vm_scan_seq.hip", "constexpr bool kChBcPairs = true;", "constexpr bool kChBcPairs = false;")],
    # persistent GEMM pricing (results wrong): no output stores
    "tg_nostore": [("vm_gemm_tile.hip", "          __builtin_amdgcn_raw_buffer_store_b128(v, o, st_lane + col * 2, 0, NORM ? kTileSC1 : 0);",
                    "          if (v[0] == 0x12345 && v[3] == 0x777) __builtin_amdgcn_raw_buffer_store_b128(v, o, st_lane + col * 2, 0, NORM ? kTileSC1 : 0);")],
    # persistent GEMM output stores with another cache policy: nt (aux 2) / sc0 (aux 1) / sc0 nt (3)
    "tg_st_nt": [("vm_gemm_tile.hip", "          __builtin_amdgcn_raw_buffer_store_b128(v, o, st_lane + col * 2, 0, NORM ? kTileSC1 : 0);", "          __builtin_amdgcn_raw_buffer_store_b128(v, o, st_lane + col * 2, 0, NORM ? kTileSC1 : 2);")],
    "tg_st_sc0": [("vm_gemm_tile.hip", "          __builtin_amdgcn_raw_buffer_store_b128(v, o, st_lane + col * 2, 0, NORM ? kTileSC1 : 0);", "          __builtin_amdgcn_raw_buffer_store_b128(v, o, st_lane + col * 2, 0, NORM ? kTileSC1 : 1);")],
    "tg_st_sc0nt": [("vm_gemm_tile.hip", "          __builtin_amdgcn_raw_buffer_store_b128(v, o, st_lane + col * 2, 0, NORM ? kTileSC1 : 0);", "          __builtin_amdgcn_raw_buffer_store_b128(v, o, st_lane + col * 2, 0, NORM ? kTileSC1 : 3);")],
    # persistent GEMM pricing (results may be wrong): the first K-tile's waits after a tile's
    # stores allow the stores as younger ops (no drain of the stores at the tile boundary)
    "tg_st_nodrain": [("vm_gemm_tile.hip", "        if constexpr (P != 2) tg_wait_vm<VM>();",
                       "        if constexpr (P != 2) { if constexpr (kt == 0) tg_wait_vm<VM + S>(); else tg_wait_vm<VM>(); }")],
    # persistent GEMM output stores sc1 (write-through, the line leaves L2) / sc0 sc1
    "tg_st_sc1": [("vm_gemm_tile.hip", "          __builtin_amdgcn_raw_buffer_store_b128(v, o, st_lane + col * 2, 0, NORM ? kTileSC1 : 0);", "          __builtin_amdgcn_raw_buffer_store_b128(v, o, st_lane + col * 2, 0, NORM ? kTileSC1 : 16);")],
    "tg_st_sc01": [("vm_gemm_tile.hip", "          __builtin_amdgcn_raw_buffer_store_b128(v, o, st_lane + col * 2, 0, NORM ? kTileSC1 : 0);", "          __builtin_amdgcn_raw_buffer_store_b128(v, o, st_lane + col * 2, 0, NORM ? kTileSC1 : 17);")],
    # persistent GEMM pricing (results wrong): every tile stages the first N-panel of W
    # (w_fixed: W L2-resident) / the first row block of x (x_fixed)
    "tg_w_fixed": [("vm_gemm_tile.hip", "    r.wsoff = nt * BN * wbytes;", "    r.wsoff = 0 * nt * BN * wbytes;")],
    "tg_x_fixed": [("vm_gemm_tile.hip", "    r.x = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(p.x + m0 * p.ldx), 0,",
                    "    r.x = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(p.x + 0 * m0 * p.ldx), 0,")],
    # persistent GEMM: the A-bottom half of a tile stored after the next tile's phase 1
    "tg_defer": [("vm_gemm_tile.hip", "constexpr bool kTileDeferStore = false;", "constexpr bool kTileDeferStore = true;")],
    # persistent GEMM: every wave stores a finished tile at the same time (no MFMA beside it)
    "tg_sync": [("vm_gemm_tile.hip", "constexpr bool kTileSyncStore = false;", "constexpr bool kTileSyncStore = true;")],
    # persistent GEMM pricing (results wrong): every tile's stores go to tile 0's rows (an
    # L2-resident 128 KB target: same instructions, no HBM write stream)
    "tg_st_l2": [("vm_gemm_tile.hip", "      m0 = static_cast<long long>(mt) * BM + r0;", "      m0 = 0 * static_cast<long long>(mt) * BM + r0;")],
    # B = 448 scan capped at 6 workgroups (3 waves per SIMD) per CU by 5 KB of padding LDS,
    # leaving a wave slot per SIMD for another stream's kernel
    "dtp_occ3": [("vm_scan_seq.hip", "    case 3: hipLaunchKernelGGL(scan_seq_dtp_kernel<3>, grid, dim3(64 * kSeqNW), 0, s, p, q); break;",
                  "    case 3: hipLaunchKernelGGL(scan_seq_dtp_kernel<3>, grid, dim3(64 * kSeqNW), 5120, s, p, q); break;")],
    # add_rms_bf16_kernel with non-temporal (nt) loads / stores
    "an_ld_nt": [("vm_norm.hip", '    const auto q = __builtin_amdgcn_raw_buffer_load_b64(xr, off(j, 2), 0, 0);\n    xq[j][0] = q[0];', '    const auto q = __builtin_amdgcn_raw_buffer_load_b64(xr, off(j, 2), 0, 2);\n    xq[j][0] = q[0];'),
                 ("vm_norm.hip", '    if constexpr (RES) rq[j] = __builtin_bit_cast(v4f, __builtin_amdgcn_raw_buffer_load_b128(rr, off(j, 4), 0, 0));', '    if constexpr (RES) rq[j] = __builtin_bit_cast(v4f, __builtin_amdgcn_raw_buffer_load_b128(rr, off(j, 4), 0, 2));')],
    "an_st_nt": [("vm_norm.hip", '    __builtin_amdgcn_raw_buffer_store_b64(o2, orr, off(j, 2), 0, 0);\n    if constexpr (RO) {', '    __builtin_amdgcn_raw_buffer_store_b64(o2, orr, off(j, 2), 0, 2);\n    if constexpr (RO) {'),
                 ("vm_norm.hip", '      __builtin_amdgcn_raw_buffer_store_b128(r4, ror, off(j, 4), 0, 0);\n    }\n  }\n}', '      __builtin_amdgcn_raw_buffer_store_b128(r4, ror, off(j, 4), 0, 2);\n    }\n  }\n}')],
    "tg_prio1": [("vm_gemm_tile.hip", "constexpr int kTilePrio = 0;", "constexpr int kTilePrio = 1;")],
    # persistent GEMM phase timestamps (scripts/diag/gemm_stamps.py)
    "tg_stamp": [("vm_gemm_tile.hip", "constexpr bool kTileStamps = false;\n\n}  // namespace\n\n__device__ void tg_stamp_sink(int idx, unsigned long long t);",
                  "constexpr bool kTileStamps = true;\n\n}  // namespace\n\n__device__ unsigned long long g_tg_stamps[1024];\n"
                  "__device__ void tg_stamp_sink(int idx, unsigned long long t) { if (idx < 1024) g_tg_stamps[idx] = t; }"),
                 ("vm_gemm_tile.hip", "#undef VM_TG_CFG\n#undef VM_TG_K\n",
                  "#undef VM_TG_CFG\n#undef VM_TG_K\n}  // namespace vm\nextern \"C\" int vm_tile_stamps(unsigned long long* host) {\n"
                  "  return hipMemcpyFromSymbol(host, HIP_SYMBOL(vm::g_tg_stamps), sizeof(vm::g_tg_stamps)) == hipSuccess ? 0 : -1;\n}\nnamespace vm {\n")],
    "tg_lgkm0": [("vm_gemm_tile.hip", "constexpr bool kTileLgkmLate = true;", "constexpr bool kTileLgkmLate = false;")],
    "tg_prio2": [("vm_gemm_tile.hip", "constexpr int kTilePrio = 0;", "constexpr int kTilePrio = 2;")],
    # dt_proj-in-scan kernel: each step's y epilogue in its own step's region (before r04)
    "dtp_yearly": [("vm_scan_seq.hip", "constexpr bool kDtpYLate = true;", "constexpr bool kDtpYLate = false;")],
    # chunked scan: 16-wave workgroups (one state per wave in the composition / hand-off,
    # 4 waves per SIMD) instead of 8
    "ch16": [("vm_scan_seq.hip", "constexpr int kChW = 8;  // segments (waves) per workgroup",
              "constexpr int kChW = 16;  // segments (waves) per workgroup")],
    # persistent GEMM: tight wait before the output stores, the next tile's first two waits
    # skipped (kTileStoreWait 1) instead of draining the stores at the next wait
    "tg_sw1": [("vm_gemm_tile.hip", "constexpr int kTileStoreWait = 0;",
                "constexpr int kTileStoreWait = 1;")],
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
    # small-M GEMM: the register-ring kernel instead of the LDS-DMA pipelined form
    "ldma_old": [("vm_gemm.hip", "constexpr bool kLinearDma = true;", "constexpr bool kLinearDma = false;")],
    # LDS-DMA GEMM tile / depth alternatives: 128x128 with three stage buffers (one
    # workgroup per CU); narrow outputs on 128x64 tiles with three buffers
    "ldma3": [("vm_gemm.hip", "  if (p.n >= 1024) VM_LDMA_TILE(128, 128, 2, 4)",
               "  if (p.n >= 1024) VM_LDMA_TILE(128, 128, 3, 2)")],
    "ldma_o64": [("vm_gemm.hip", "  else VM_LDMA_TILE(128, 64, 3, 4)",
                  "  else VM_LDMA_TILE(64, 64, 3, 2)")],
    "ldma_o2": [("vm_gemm.hip", "  else VM_LDMA_TILE(128, 64, 3, 4)",
                 "  else VM_LDMA_TILE(64, 64, 2, 2)")],
    # LDS-DMA GEMM tile alternatives for in_proj (N >= 1024) and out_proj at B = 1
    "ldma_i128x64": [("vm_gemm.hip", "  if (p.n >= 1024) VM_LDMA_TILE(128, 128, 2, 4)",
                      "  if (p.n >= 1024) VM_LDMA_TILE(128, 64, 3, 2)")],
    # wide conv_proj occupancy probe: LDS padded so 2 (cp_occ2) workgroups fit per CU instead of 3
    "cp_occ2": [("vm_conv_proj.hip", "  const size_t lds = static_cast<size_t>(dim) * 5 * sizeof(float);",
                 "  const size_t lds = static_cast<size_t>(dim) * 5 * sizeof(float) + 30000;")],
    # final norm + pooling through the dtype-generic rows kernel only
    "np_generic": [("vm_norm.hip", "constexpr bool kPoolFast = true;", "constexpr bool kPoolFast = false;")],
    "ldma16_i128x128": [("vm_gemm.hip", "  if (p.n >= 1024) VM_LDMA_TILE(128, 128, 2, 4)",
                         "  if (p.n >= 1024) VM_LDMA_TILE(128, 128, 2, 8)")],
    "ldma8_i64x128": [("vm_gemm.hip", "  if (p.n >= 1024) VM_LDMA_TILE(128, 128, 2, 4)",
                       "  if (p.n >= 1024) VM_LDMA_TILE(64, 128, 2, 4)")],
    # fused small-batch conv_proj pricing (results wrong): W_x fragments from an out-of-range
    # offset (no traffic) / no x_proj MFMA / no u stores
    "cf_nowx": [("vm_conv_proj_sk.hip",
                 "                      wxr, opaque(kc < nch ? ((j * 16 + (lane & 15)) * p.dim + c0 + kc) * 2 : kOut),",
                 "                      wxr, opaque(kOut + 0 * kc),")],
    "cf_nomfma": [("vm_conv_proj_sk.hip",
                   "      acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, wv[ks][j], acc[j], 0, 0, 0);\n  }\n  // u rows leave",
                   "      acc[j][0] += av[0] + wv[ks][j][0];\n  }\n  // u rows leave")],
    "cf_nou": [("vm_conv_proj_sk.hip",
                "        opaque(ch < nch && tok0 + row < ntok ? ((tok0 + row) * static_cast<int>(p.u_tl) + c0 + ch) * 2\n                                             : kOut),",
                "        opaque(kOut + 0 * ch),")],
    # fused small-batch conv_proj with XCD-contiguous token tiles (the in_proj GEMM's row runs)
    "cf_xcd": [("vm_conv_proj_sk.hip", "  const int tok0 = blockIdx.x * kFuTok;",
                "  const int tok0 = [] { const int nwg = gridDim.x, h = blockIdx.x, x = h & 7, q = nwg >> 3, r = nwg & 7;"
                " return ((x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (h >> 3)) * kFuTok; }();")],
    # eight-wave (4 x 2) forms at one workgroup per CU (round 4)
    "ldma8_i256x128": [("vm_gemm.hip", "  if (p.n >= 1024) VM_LDMA_TILE(128, 128, 2, 4)",
                        "  if (p.n >= 1024) VM_LDMA_TILE(256, 128, 2, 4)")],
    "ldma8_i256x128b3": [("vm_gemm.hip", "  if (p.n >= 1024) VM_LDMA_TILE(128, 128, 2, 4)",
                          "  if (p.n >= 1024) VM_LDMA_TILE(256, 128, 3, 4)")],
    "ldma8_i128x128": [("vm_gemm.hip", "  if (p.n >= 1024) VM_LDMA_TILE(128, 128, 2, 4)",
                        "  if (p.n >= 1024) VM_LDMA_TILE(128, 128, 2, 4)")],
    "ldma8_i128x128b3": [("vm_gemm.hip", "  if (p.n >= 1024) VM_LDMA_TILE(128, 128, 2, 4)",
                          "  if (p.n >= 1024) VM_LDMA_TILE(128, 128, 3, 4)")],
    "ldma8_i128x256": [("vm_gemm.hip", "  if (p.n >= 1024) VM_LDMA_TILE(128, 128, 2, 4)",
                        "  if (p.n >= 1024) VM_LDMA_TILE(128, 256, 2, 4)")],
    "ldma16_i256x128": [("vm_gemm.hip", "  if (p.n >= 1024) VM_LDMA_TILE(128, 128, 2, 4)",
                         "  if (p.n >= 1024) VM_LDMA_TILE(256, 128, 2, 8)")],
    "ldma16_i128x128b3": [("vm_gemm.hip", "  if (p.n >= 1024) VM_LDMA_TILE(128, 128, 2, 4)",
                           "  if (p.n >= 1024) VM_LDMA_TILE(128, 128, 3, 8)")],
    "ldma16_o128x64": [("vm_gemm.hip", "  else VM_LDMA_TILE(128, 64, 3, 4)",
                        "  else VM_LDMA_TILE(128, 64, 3, 8)")],
    "ldma8_o128x64b2": [("vm_gemm.hip", "  else VM_LDMA_TILE(128, 64, 3, 4)",
                         "  else VM_LDMA_TILE(128, 64, 2, 4)")],
    "ldma8_o128x64": [("vm_gemm.hip", "  else VM_LDMA_TILE(128, 64, 3, 4)",
                       "  else VM_LDMA_TILE(128, 64, 3, 4)")],
    "ldma8_o128x64b4": [("vm_gemm.hip", "  else VM_LDMA_TILE(128, 64, 3, 4)",
                         "  else VM_LDMA_TILE(128, 64, 4, 4)")],
    "ldma_i256x128": [("vm_gemm.hip", "  if (p.n >= 1024) VM_LDMA_TILE(128, 128, 2, 4)",
                       "  if (p.n >= 1024) VM_LDMA_TILE(256, 128, 2, 2)")],
    "ldma_i128x256": [("vm_gemm.hip", "  if (p.n >= 1024) VM_LDMA_TILE(128, 128, 2, 4)",
                       "  if (p.n >= 1024) VM_LDMA_TILE(128, 256, 2, 2)")],
    "ldma_i64x128": [("vm_gemm.hip", "  if (p.n >= 1024) VM_LDMA_TILE(128, 128, 2, 4)",
                      "  if (p.n >= 1024) VM_LDMA_TILE(64, 128, 3, 2)")],
    "ldma_o64n4": [("vm_gemm.hip", "  else VM_LDMA_TILE(128, 64, 3, 4)",
                    "  else VM_LDMA_TILE(64, 64, 4, 2)")],
    # one-launch chunked scan: the preceding blocks' flags polled one after another by
    # thread 0 (the round-2 form) instead of in parallel by wave 0
    "poll_serial": [("vm_scan_seq.hip", "        for (int j = lane; j < blk; j += 64)",
                     "        for (int j = 0; lane == 0 && j < blk; ++j)")],
    # fused small-batch conv_proj with full __syncthreads() (vmcnt(0) drains) at its barriers
    "cp_sync": [("vm_conv_proj_sk.hip", """__device__ __forceinline__ void fu_lds_barrier() {
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
  __builtin_amdgcn_s_barrier();""", """__device__ __forceinline__ void fu_lds_barrier() {
  __syncthreads();""")],
    # phase timestamps of the fused small-batch conv_proj (s_memrealtime, 100 MHz) per
    # workgroup into a device array read back by vm_dbg_read_stamps
    # (scripts/diag/stamp_conv_proj.py); results unchanged
    "cp_stamp": [
        ("vm_conv_proj_sk.hip", "template <int NB, bool CS32>  // NB = e_pad / 16 x_proj column blocks; CS32: fp32 conv state in",
         "__device__ unsigned long long vm_dbg_stamps[4096 * 8];\n"
         "#define VM_STAMP(K) __builtin_amdgcn_sched_barrier(0); if (threadIdx.x == 0) vm_dbg_stamps[blockIdx.x * 8 + (K)] = __builtin_amdgcn_s_memrealtime(); __builtin_amdgcn_sched_barrier(0);\n"
         "template <int NB, bool CS32>  // NB = e_pad / 16 x_proj column blocks; CS32: fp32 conv state in"),
        ("vm_conv_proj_sk.hip", "  const int ntok = q.ntok;\n\n  // Every global load and store",
         "  const int ntok = q.ntok;\n  VM_STAMP(0)\n\n  // Every global load and store"),
        ("vm_conv_proj_sk.hip", "  // ---- new conv state of a sequence ending in this tile: its last W raw inputs ----",
         "  VM_STAMP(1)\n  // ---- new conv state of a sequence ending in this tile: its last W raw inputs ----"),
        ("vm_conv_proj_sk.hip", "  fu_lds_barrier();  // every wave's u tile is consumed: the area becomes the partials",
         "  fu_lds_barrier();  // every wave's u tile is consumed: the area becomes the partials\n  VM_STAMP(2)"),
        ("vm_conv_proj_sk.hip", "  if (!do_dt) return;\n  fu_lds_barrier();\n  // ---- dt for channels",
         "  VM_STAMP(3)\n  if (!do_dt) return;\n  fu_lds_barrier();\n  // ---- dt for channels"),
        ("vm_conv_proj_sk.hip", "  fu_lds_barrier();\n  // 16 token rows x dim channels out, 16 B per lane-store",
         "  fu_lds_barrier();\n  VM_STAMP(4)\n  // 16 token rows x dim channels out, 16 B per lane-store"),
        ("vm_conv_proj_sk.hip", "          *reinterpret_cast<const uint4*>(&sDT[t * dtp + qd * 8]);\n  }\n}",
         "          *reinterpret_cast<const uint4*>(&sDT[t * dtp + qd * 8]);\n  }\n  __builtin_amdgcn_s_waitcnt(0);\n  __syncthreads();\n  VM_STAMP(5)\n}"),
        ("vm_conv_proj_sk.hip", "bool conv_proj_fused_ok(const ConvProjTmArgs& a) {",
         "}  // namespace vm\nextern \"C\" int vm_dbg_read_stamps(void* dst) {\n"
         "  return static_cast<int>(hipMemcpyFromSymbol(dst, HIP_SYMBOL(vm::vm_dbg_stamps), sizeof(vm::vm_dbg_stamps)));\n}\n"
         "namespace vm {\nbool conv_proj_fused_ok(const ConvProjTmArgs& a) {"),
    ],
    # phase timestamps of the one-launch chunked scan (PASS 3) per workgroup: entry (0),
    # start-up loads landed (1), PASS 1 steps done (2), segments composed and aggregate
    # granules stored (3), PASS 2 prefetch issued (4), preceding granules seen and entry
    # state composed (5), PASS 2 done and drained (6)
    # (scripts/diag/stamp_scan.py); results unchanged
    "sc_stamp": [
        ("vm_scan_seq.hip", "template <typename T, int PASS, bool SP, bool HZ, bool BC1, bool PAIR, bool DTP = false>\n__global__ __launch_bounds__(64 * kChW)",
         "__device__ unsigned long long vm_dbg_stamps[4096 * 8];\n"
         "#define VM_STAMP(K) __builtin_amdgcn_sched_barrier(0); if (PASS == 3 && threadIdx.x == 0) vm_dbg_stamps[(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z)) * 8 + (K)] = __builtin_amdgcn_s_memrealtime(); __builtin_amdgcn_sched_barrier(0);\n"
         "template <typename T, int PASS, bool SP, bool HZ, bool BC1, bool PAIR, bool DTP = false>\n__global__ __launch_bounds__(64 * kChW)"),
        ("vm_scan_seq.hip", "  f2 A2[kMaxN / 2], h[kMaxN / 2];\n#pragma unroll\n  for (int q = 0; q < kMaxN / 2; ++q) {\n    A2[q] = f2{sA[2 * q][lane], sA[2 * q + 1][lane]};",
         "  VM_STAMP(7)\n  f2 A2[kMaxN / 2], h[kMaxN / 2];\n#pragma unroll\n  for (int q = 0; q < kMaxN / 2; ++q) {\n    A2[q] = f2{sA[2 * q][lane], sA[2 * q + 1][lane]};"),
        ("vm_scan_seq.hip", "  const int nch = min(64, p.dim - d0);  // live channels of this group\n",
         "  const int nch = min(64, p.dim - d0);  // live channels of this group\n  VM_STAMP(0)\n"),
        ("vm_scan_seq.hip", "  // pending they would merge into the step loop's header waits\n  __builtin_amdgcn_s_waitcnt(0);\n",
         "  // pending they would merge into the step loop's header waits\n  __builtin_amdgcn_s_waitcnt(0);\n  VM_STAMP(1)\n"),
        ("vm_scan_seq.hip", "  run_steps(BoolTag<false>{});\n#pragma unroll\n",
         "  run_steps(BoolTag<false>{});\n  VM_STAMP(2)\n#pragma unroll\n"),
        ("vm_scan_seq.hip", "    // every wave's E_j is in sH (an LDS-only barrier: the granule stores need no drain)",
         "    VM_STAMP(3)\n    // every wave's E_j is in sH (an LDS-only barrier: the granule stores need no drain)"),
        ("vm_scan_seq.hip", "    // ---- walk the preceding blocks' aggregates from h0 to this block's entry ----\n    // Wave w",
         "    VM_STAMP(4)\n    // ---- walk the preceding blocks' aggregates from h0 to this block's entry ----\n    // Wave w"),
        ("vm_scan_seq.hip", "    run_steps(BoolTag<true>{});\n    finish();\n    if (tid == 0) {  // count this block out",
         "    VM_STAMP(5)\n    run_steps(BoolTag<true>{});\n    finish();\n    __builtin_amdgcn_s_waitcnt(0);\n    __syncthreads();\n    VM_STAMP(6)\n    if (tid == 0) {  // count this block out"),
        ("vm_scan_seq.hip", "bool seq_supported(const ScanParams& p, int dtype) {",
         "}  // namespace vm\nextern \"C\" int vm_dbg_read_stamps(void* dst) {\n"
         "  return static_cast<int>(hipMemcpyFromSymbol(dst, HIP_SYMBOL(vm::vm_dbg_stamps), sizeof(vm::vm_dbg_stamps)));\n}\n"
         "namespace vm {\nbool seq_supported(const ScanParams& p, int dtype) {"),
    ],
    # per-WAVE timestamps of the one-launch chunked scan (lane 0 of each wave, s_memrealtime):
    # 0 start-up wait passed, 1 dt block + A2 ready, 2 PASS 1 loop done, 3 after the
    # compose barrier + granule stores (scripts/diag/stamp_scan_waves.py); results unchanged
    "sc_stampw": [
        ("vm_scan_seq.hip", "template <typename T, int PASS, bool SP, bool HZ, bool BC1, bool PAIR, bool DTP = false>\n__global__ __launch_bounds__(64 * kChW)",
         "__device__ unsigned long long vm_dbg_stamps[4096 * 8 * 4];\n"
         "#define VM_STAMPW(K) __builtin_amdgcn_sched_barrier(0); if (PASS == 3 && (threadIdx.x & 63) == 0) vm_dbg_stamps[((blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z)) * 8 + (threadIdx.x >> 6)) * 4 + (K)] = __builtin_amdgcn_s_memrealtime(); __builtin_amdgcn_sched_barrier(0);\n"
         "template <typename T, int PASS, bool SP, bool HZ, bool BC1, bool PAIR, bool DTP = false>\n__global__ __launch_bounds__(64 * kChW)"),
        ("vm_scan_seq.hip", '  asm volatile("" ::"v"(warm[0]), "v"(warm[1]));  // the L2 warm-up loads are not dead',
         '  asm volatile("" ::"v"(warm[0]), "v"(warm[1]));  // the L2 warm-up loads are not dead\n  VM_STAMPW(0)'),
        ("vm_scan_seq.hip", "  f2 A2[kMaxN / 2], h[kMaxN / 2];\n#pragma unroll\n  for (int q = 0; q < kMaxN / 2; ++q) {\n    A2[q] = f2{sA[2 * q][lane], sA[2 * q + 1][lane]};",
         "  VM_STAMPW(1)\n  f2 A2[kMaxN / 2], h[kMaxN / 2];\n#pragma unroll\n  for (int q = 0; q < kMaxN / 2; ++q) {\n    A2[q] = f2{sA[2 * q][lane], sA[2 * q + 1][lane]};"),
        ("vm_scan_seq.hip", "  run_steps(BoolTag<false>{});\n", "  run_steps(BoolTag<false>{});\n  VM_STAMPW(2)\n"),
        ("vm_scan_seq.hip", "    // every wave's E_j is in sH (an LDS-only barrier: the granule stores need no drain)",
         "    VM_STAMPW(3)\n    // every wave's E_j is in sH (an LDS-only barrier: the granule stores need no drain)"),
        ("vm_scan_seq.hip", "bool seq_supported(const ScanParams& p, int dtype) {",
         "}  // namespace vm\nextern \"C\" int vm_dbg_read_stamps(void* dst) {\n"
         "  return static_cast<int>(hipMemcpyFromSymbol(dst, HIP_SYMBOL(vm::vm_dbg_stamps), sizeof(vm::vm_dbg_stamps)));\n}\n"
         "namespace vm {\nbool seq_supported(const ScanParams& p, int dtype) {"),
    ],
    # per-wave phase timestamps of the fused small-batch conv_proj (lane 0 of every wave):
    # entry (0), conv done (1), W_x 2-3 issued (2), u LDS tile written (3), x_proj MFMAs
    # retired (4), u rows stored (5), W_dt issued (6), barrier passed (7)
    # (scripts/diag/stamp_conv_proj.py --waves); results unchanged
    "cp_stampw": [
        ("vm_conv_proj_sk.hip", "template <int NB, bool CS32>  // NB = e_pad / 16 x_proj column blocks; CS32: fp32 conv state in",
         "__device__ unsigned long long vm_dbg_stamps[2048 * 16 * 8];\n"
         "#define VM_STAMP(K) __builtin_amdgcn_sched_barrier(0); if ((threadIdx.x & 63) == 0) vm_dbg_stamps[(blockIdx.x * 16 + (threadIdx.x >> 6)) * 8 + (K)] = __builtin_amdgcn_s_memrealtime(); __builtin_amdgcn_sched_barrier(0);\n"
         "template <int NB, bool CS32>  // NB = e_pad / 16 x_proj column blocks; CS32: fp32 conv state in"),
        ("vm_conv_proj_sk.hip", "  const int ntok = q.ntok;\n\n  // Every global load and store",
         "  const int ntok = q.ntok;\n  VM_STAMP(0)\n\n  // Every global load and store"),
        ("vm_conv_proj_sk.hip", "  wx_load(2);\n  wx_load(3);\n", "  VM_STAMP(1)\n  wx_load(2);\n  wx_load(3);\n  VM_STAMP(2)\n"),
        ("vm_conv_proj_sk.hip", "  __builtin_amdgcn_wave_barrier();\n  // ---- x_proj partial",
         "  VM_STAMP(3)\n  __builtin_amdgcn_wave_barrier();\n  // ---- x_proj partial"),
        ("vm_conv_proj_sk.hip", "  // u rows leave from the LDS tile as 16-byte pieces",
         "  { float sink = 0.0f;\n#pragma unroll\n    for (int j = 0; j < NB; ++j) sink += acc[j][0];\n    asm volatile(\"\" :: \"v\"(sink)); }\n  VM_STAMP(4)\n  // u rows leave from the LDS tile as 16-byte pieces"),
        ("vm_conv_proj_sk.hip", "  // W_dt fragments for this wave's dt channels (128 per wave",
         "  VM_STAMP(5)\n  // W_dt fragments for this wave's dt channels (128 per wave"),
        ("vm_conv_proj_sk.hip", "  fu_lds_barrier();  // every wave's u tile is consumed: the area becomes the partials",
         "  VM_STAMP(6)\n  fu_lds_barrier();  // every wave's u tile is consumed: the area becomes the partials\n  VM_STAMP(7)"),
        ("vm_conv_proj_sk.hip", "bool conv_proj_fused_ok(const ConvProjTmArgs& a) {",
         "}  // namespace vm\nextern \"C\" int vm_dbg_read_stamps(void* dst) {\n"
         "  return static_cast<int>(hipMemcpyFromSymbol(dst, HIP_SYMBOL(vm::vm_dbg_stamps), sizeof(vm::vm_dbg_stamps)));\n}\n"
         "namespace vm {\nbool conv_proj_fused_ok(const ConvProjTmArgs& a) {"),
    ],
    # timing probe: every step reads the segment's first B/C row (L1/K$-resident), so the
    # chunk kernel's time without the per-step scalar-load latency shows (results wrong)
    "bc_fixed": [("vm_scan_seq.hip",
                  "      bc_load(min(t + 1, tlast), bcw[(j + 1) & 1]);",
                  "      bc_load(t_beg, bcw[(j + 1) & 1]);")],
    # B = 1 patch kernel (patch_mfma16_kernel) cost split: two k-steps only / no
    # positional loads in the epilogue / no head+pad rows (results wrong)
    "pt_k2": [("vm_patch.hip", "  for (int kk = 0; kk < p.K; kk += 64) {\n    load(kk + 32, a1, b1);",
               "  for (int kk = 0; kk < 64; kk += 64) {\n    load(kk + 32, a1, b1);")],
    "pt_noepi": [("vm_patch.hip",
                  "    svs[it] = *reinterpret_cast<const uint4*>(spos + (long long)sp * p.embed + n);\n"
                  "    tvs[it] = *reinterpret_cast<const uint4*>(tpos + (long long)t * p.embed + n);\n"
                  "    orow[it] = ok ? b * p.out_sb + (long long)(p.row0 + rem) * p.embed + n : -1;\n"
                  "    soff[it] = ml * (kPN + 8) + c8;",
                  "    svs[it] = make_uint4(sp, 0, 0, 0);\n    tvs[it] = make_uint4(t, 0, 0, 0);\n"
                  "    orow[it] = ok ? b * p.out_sb + (long long)(p.row0 + rem) * p.embed + n : -1;\n"
                  "    soff[it] = ml * (kPN + 8) + c8;")],

    # the B = 1 patch kernel returning at once (the launch + event floor) / two k-steps and
    # no output stores (results wrong)
    "pt_empty": [("vm_patch.hip", "  __shared__ __attribute__((aligned(16))) bf16_t stile[kPT * (kPN + 8)];\n  const int tid = threadIdx.x;",
                  "  __shared__ __attribute__((aligned(16))) bf16_t stile[kPT * (kPN + 8)];\n  if (p.M > 0) return;\n  const int tid = threadIdx.x;")],
    "pt_k2_nost": [("vm_patch.hip", "  for (int kk = 0; kk < p.K; kk += 64) {\n    load(kk + 32, a1, b1);",
                    "  for (int kk = 0; kk < 64; kk += 64) {\n    load(kk + 32, a1, b1);"),
                   ("vm_patch.hip", "    *reinterpret_cast<uint4*>(out + orow[it]) = make_uint4(ow[0], ow[1], ow[2], ow[3]);\n  }\n  patch_frame_rows<bf16_t>(p, blockIdx.x, gridDim.x, blockIdx.y);",
                    "    if (ow[0] == 0x12345678u) *reinterpret_cast<uint4*>(out + orow[it]) = make_uint4(ow[0], ow[1], ow[2], ow[3]);\n  }\n  patch_frame_rows<bf16_t>(p, blockIdx.x, gridDim.x, blockIdx.y);")],

    # the token-major dtp scan's waves at raised issue priority (s_setprio), so that beside
    # another sub-batch stream's memory-bound kernels on the same SIMD its instructions
    # issue first
    "dtp_prio2": [("vm_scan_seq.hip", "  int gx = blockIdx.x, gy = blockIdx.y, gz = blockIdx.z;\n  xcd_order(gx, gy, gz);",
                   "  __builtin_amdgcn_s_setprio(2);\n  int gx = blockIdx.x, gy = blockIdx.y, gz = blockIdx.z;\n  xcd_order(gx, gy, gz);")],
    "dtp_prio3": [("vm_scan_seq.hip", "  int gx = blockIdx.x, gy = blockIdx.y, gz = blockIdx.z;\n  xcd_order(gx, gy, gz);",
                   "  __builtin_amdgcn_s_setprio(3);\n  int gx = blockIdx.x, gy = blockIdx.y, gz = blockIdx.z;\n  xcd_order(gx, gy, gz);")],

    # add + RMSNorm (the B = 448 form) / the wide conv_proj at raised wave priority, so that
    # beside the other sub-batch's VALU-bound scan their memory requests issue first
    "an_prio3": [("vm_norm.hip", "void add_rms_bf16_kernel(const NormParams p) {\n",
                  "void add_rms_bf16_kernel(const NormParams p) {\n  __builtin_amdgcn_s_setprio(3);\n")],
    "cp_prio3": [("vm_conv_proj.hip", "void conv_proj_kernel(const ConvProjParams p) {\n",
                  "void conv_proj_kernel(const ConvProjParams p) {\n  __builtin_amdgcn_s_setprio(3);\n")],
    # in_proj + conv epilogue pricing (results wrong): x tiles stop after the LDS tile
    # (ic_noepi), skip the conv + u stores (ic_noconv), skip the x_proj MFMA + partial
    # stores (ic_nopart)
    "ic_noepi": [("vm_inproj_conv.hip", "  if (!xt) {  // ---- z tile", "  if (xt) return;\n  if (!xt) {  // ---- z tile")],
    "ic_noconv": [("vm_inproj_conv.hip", "  uint32_t upk[kRows];\n#pragma unroll\n  for (int i = 0; i < kRows; ++i) {\n    float al",
                   "  uint32_t upk[kRows];\n#pragma unroll\n  for (int i = 0; i < kRows && tok_lo < -100; ++i) {\n    float al"),
                  ("vm_inproj_conv.hip", "    if (st < 3) {  // uniform", "    upk[i] = xw[i];\n    if (st < 3 && tok_lo < -100) {  // uniform"),
                  ("vm_inproj_conv.hip", "    if (tok < q.ntok) *reinterpret_cast<uint32_t*>(p.u", "    if (tok < -5) *reinterpret_cast<uint32_t*>(p.u")],
    "ic_nopart": [("vm_inproj_conv.hip", "  const bool mw = wave < kIcOut / 16;", "  if (tok_lo >= 0) return;\n  const bool mw = wave < kIcOut / 16;")],
    # ... no u global stores (ic_nou), no partial global stores (ic_nops), z tiles skipped
    # (ic_noz), no conv-state / new-conv-state work (ic_nocs)
    "ic_nou": [("vm_inproj_conv.hip", "    if (tok < q.ntok) *reinterpret_cast<uint32_t*>(p.u", "    if (tok < -5) *reinterpret_cast<uint32_t*>(p.u")],
    "ic_nops": [("vm_inproj_conv.hip", "      if (tok < q.ntok)\n        *reinterpret_cast<float4*>(q.part", "      if (tok < -5)\n        *reinterpret_cast<float4*>(q.part")],
    "ic_noz": [("vm_inproj_conv.hip", "  const int m0 = xt ? rt * kIcOut - kIcHalo : rt * 128;", "  if (!xt) return;\n  const int m0 = xt ? rt * kIcOut - kIcHalo : rt * 128;")],
    # in_proj + conv epilogue phase stamps (scripts/diag/inproj_conv_stamps.py): wave 0 of every
    # workgroup records s_memrealtime at 8 points into g_ic_stamps[workgroup][8]
    "ic_stamp": [
        ("vm_inproj_conv.hip", "template <int NK, int NB>\n__global__ __launch_bounds__(512) void inproj_conv_kernel(",
         "__device__ unsigned long long g_ic_stamps[4096 * 8];\n#define IC_ST(P) do { if (tid == 0 && blockIdx.x < 4096) g_ic_stamps[blockIdx.x * 8 + (P)] = __builtin_amdgcn_s_memrealtime(); } while (0)\n"
         "template <int NK, int NB>\n__global__ __launch_bounds__(512) void inproj_conv_kernel("),
        ("vm_inproj_conv.hip", "  const int wm = wave >> 1, wn = wave & 1;\n", "  const int wm = wave >> 1, wn = wave & 1;\n  IC_ST(0);\n"),
        ("vm_inproj_conv.hip", "  __syncthreads();  // every wave is past its last fragment reads\n", "  __syncthreads();  // every wave is past its last fragment reads\n  IC_ST(1);\n"),
        ("vm_inproj_conv.hip", "  // ---- x tile epilogue ----\n", "  // ---- x tile epilogue ----\n  IC_ST(2);\n"),
        ("vm_inproj_conv.hip", "  // conv + SiLU: channels c, c + 1 (one packed word)", "  IC_ST(3);\n  // conv + SiLU: channels c, c + 1 (one packed word)"),
        ("vm_inproj_conv.hip", "  __syncthreads();  // every wave is past its reads of the x tile: u takes its rows\n", "  IC_ST(4);\n  __syncthreads();  // every wave is past its reads of the x tile: u takes its rows\n"),
        ("vm_inproj_conv.hip", "  __syncthreads();  // the u / W_x tiles are free", "  IC_ST(5);\n  __syncthreads();  // the u / W_x tiles are free"),
        ("vm_inproj_conv.hip", "  __builtin_amdgcn_wave_barrier();\n  if (mw) {\n    const int nq", "  IC_ST(6);\n  __builtin_amdgcn_wave_barrier();\n  if (mw) {\n    const int nq"),
        ("vm_inproj_conv.hip", "}  // namespace vm\n\nusing namespace vm;\n",
         "}  // namespace vm\n\nusing namespace vm;\nextern \"C\" int vm_ic_stamps(unsigned long long* host) {\n"
         "  return hipMemcpyFromSymbol(host, HIP_SYMBOL(vm::g_ic_stamps), sizeof(vm::g_ic_stamps)) == hipSuccess ? 0 : -1;\n}\n")],
    # ... x tiles at raised wave priority (ic_prio), no XCD renumbering in either part (ic_norenum)
    "ic_prio": [("vm_inproj_conv.hip", "  const int m0 = xt ? rt * kIcOut - kIcHalo : rt * 128;", "  if (xt) __builtin_amdgcn_s_setprio(2);\n  const int m0 = xt ? rt * kIcOut - kIcHalo : rt * 128;")],
    "ic_norenum": [("vm_inproj_conv.hip", "  const int lt = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (h >> 3);",
                    "  const int lt = h + 0 * (xcd + qq + rr + nwg);")],
    # add + RMSNorm with 8 / 4 / 16 rows per wave at >= 2^20 rows (round 6, measured no gain
    # in the 1344-clip step, profiles/r06k_add_norm_rows_per_wave_step_ab.jsonl): the product
    # sources of commit bb2e338 (python build_variant.py --rev bb2e338 NAME)
    "ancp_prio3": [("vm_norm.hip", "void add_rms_bf16_kernel(const NormParams p) {\n",
                    "void add_rms_bf16_kernel(const NormParams p) {\n  __builtin_amdgcn_s_setprio(3);\n"),
                   ("vm_conv_proj.hip", "void conv_proj_kernel(const ConvProjParams p) {\n",
                    "void conv_proj_kernel(const ConvProjParams p) {\n  __builtin_amdgcn_s_setprio(3);\n")],

}


# Variants whose toggles left the product sources after round 5 (no untested
# path compiled into a product kernel): they patch the round-5 head's sources instead.
LEGACY_REV = "45fb10e"
LEGACY = {"ch_xcd", "dtp_d16", "tg_split", "tg_defer", "tg_sync", "tg_prio1", "tg_prio2",
          "tg_stamp", "tg_lgkm0", "tg_sw1", "tg_st_nodrain"}


def build(name, rev=None):
    if rev is None and name in LEGACY:
        rev = LEGACY_REV
    src = os.path.join(ROOT, "videomamba_amd", "csrc")
    work = os.path.join(ROOT, "build", "var", name, "src", "csrc")  # ../../include resolves
    shutil.rmtree(work, ignore_errors=True)
    shutil.copytree(src, work)
    if rev:  # the csrc sources of a git revision (e.g. HEAD: the committed baseline)
        for f in os.listdir(work):
            blob = subprocess.run(["git", "-C", ROOT, "show", f"{rev}:videomamba_amd/csrc/{f}"],
                                  capture_output=True)
            if blob.returncode == 0:
                open(os.path.join(work, f), "wb").write(blob.stdout)
    inc = os.path.join(ROOT, "build", "var", name, "include")
    shutil.rmtree(inc, ignore_errors=True)
    shutil.copytree(os.path.join(ROOT, "include"), inc)
    for fname, old, new in VARIANTS[name]:
        p = os.path.join(work, fname)
        s = open(p).read()
        assert s.count(old) >= 1, (name, fname, old)
        open(p, "w").write(s.replace(old, new))
    # VARIANT_DIR=ab puts the build where gpurun pushes it (tools/probes/var is not pushed)
    out = os.path.join(ROOT, "tools", "probes", os.environ.get("VARIANT_DIR", "var"), name)
    os.makedirs(out, exist_ok=True)
    subprocess.check_call(["make", "-C", work, "-j8", f"OUT={out}/libvideomamba_hip.so",
                           f"BUILD={os.path.join(ROOT, 'build', 'var', name, 'obj')}"])


VARIANTS["wt_all"] = VARIANTS["wt_ic"] + VARIANTS["wt_rest"]


if __name__ == "__main__":
    # python build_variant.py name...            variants of the working-tree sources
    # python build_variant.py --rev REV name     the sources of git revision REV (as "name")
    args = sys.argv[1:]
    if args and args[0] == "--rev":
        VARIANTS.setdefault(args[2], [])
        build(args[2], rev=args[1])
    else:
        for n in args:
            build(n)
