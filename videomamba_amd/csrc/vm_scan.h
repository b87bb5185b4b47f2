// Shared declarations of the selective-scan kernels (vm_scan.hip: channel-major,
// time-parallel kernels; vm_scan_seq.hip: token-major, channel-per-lane kernels).
#pragma once

#include "vm_common.h"

namespace vm {

constexpr int kMaxN = 16;

// Every (batch, channel|state, step) operand carries three element strides; the
// channel-major kernels require the step stride to be 1, the token-major ones require the
// channel (state) stride to be 1.
struct ScanParams {
  const void* u; const void* delta; const float* A; const void* B; const void* C;
  const float* D; const void* z; const float* dbias;
  const void* h0; void* hl; void* out;
  long long u_sb, u_sd, dl_sb, dl_sd, b_sb, b_sn, c_sb, c_sn, z_sb, z_sd, o_sb, o_sd;
  long long u_sl, dl_sl, b_sl, c_sl, z_sl, o_sl;
  long long h0_sb, h0_sd, hl_sb, hl_sd;
  int batch, dim, seqlen, out_len, dstate, softplus, h0_dtype, hl_dtype;
  int vec_x;   // u/delta/z/out rows allow 8-element vector access
  int vec_bc;  // B/C rows allow 8-element vector access
  // Paired scan (vm_selective_scan_bidir_fwd): batch rows b >= split take A_hi / D_hi /
  // dbias_hi and store step t's output at row ro_c0 + ro_s*t - ro_c1*umulhi(t, ro_m), the
  // frame-order reversal.  split == batch for a plain scan.
  // Their entry / last states are h0_hi / hl_hi at row b - split (same dtypes and strides).
  int split;
  const float* A_hi; const float* D_hi; const float* dbias_hi;
  const void* h0_hi; void* hl_hi;
  int ro_c0, ro_s, ro_c1; unsigned ro_m;
};

// Parameter set of batch row b (uniform per workgroup).  PAIR = false folds to the plain
// scan's (p.A, p.D, p.dbias, identity row map) at compile time.
struct PairSel {
  const float* A; const float* D; const float* dbias;
  const void* h0; void* hl; int hb;  // state pointers and the state row of this batch row
  int c0, s, c1; unsigned m;
  __device__ __forceinline__ int orow(int t) const {
    return c0 + s * t - c1 * static_cast<int>(__umulhi(static_cast<unsigned>(t), m));
  }
};
template <bool PAIR>
__device__ __forceinline__ PairSel pair_sel(const ScanParams& p, int b) {
  if (PAIR && b >= p.split)
    return {p.A_hi, p.D_hi, p.dbias_hi, p.h0_hi, p.hl_hi, b - p.split,
            p.ro_c0, p.ro_s, p.ro_c1, p.ro_m};
  return {p.A, p.D, p.dbias, p.h0, p.hl, b, 0, 1, 0, 0u};
}


// Token-major path (vm_scan_seq.hip).  Workspace for the time-segmented form, in bytes;
// 0 when the single-pass form is chosen.  `segments` receives the chosen segment count.
// segments: 0 = cost model, > 0 forced.  cus: the CU count the cost model sizes for
// (0 = the current device's; kCalibCUs = 256 when no device can be queried).
size_t seq_workspace_bytes(int batch, int dim, int seqlen, int segments, int* chosen,
                           int cus = 0);
// Launch; `workspace` must hold seq_workspace_bytes() (or be larger).  Returns false when
// the operands do not fit the token-major kernels (the caller reports the error).
bool seq_supported(const ScanParams& p, int dtype);
void seq_launch(const ScanParams& p, int dtype, int segments, void* workspace,
                size_t workspace_bytes, void* sync, size_t sync_bytes, hipStream_t s);
// Bytes of the zeroed sync buffer the one-launch chunked form needs (0: single pass).
// Word 0 is the sticky error word (non-zero after a launch whose block handoff timed out;
// vm_selective_scan_sync_status), word 1 the epoch, word 2 the launch's start count, word 3
// pad, then the {tag, value} hand-off granules.
constexpr int kSyncHeaderWords = 4;
size_t seq_sync_bytes(int batch, int dim, int seqlen, int segments, int cus = 0);
// Paired scans need the scalar-B/C kernels and, when segmented, the chunked form.
bool seq_pair_supported(const ScanParams& p, int dtype, int segments, size_t workspace_bytes);

// dt_proj folded into the single-pass token-major scan (vm_selective_scan_dtproj_fwd):
// delta = bf16(dt_low @ W_dt^T) computed per 16-step block on the matrix cores.
struct DtpArgs {
  const bf16_t* dtl;  // dt_low = the first dt_rank columns of the x_dbl rows
  long long dtl_sb;   // batch stride (elements)
  long long dtl_sl;   // row (step) stride (elements)
  const bf16_t* wdt;  // W_dt padded: (dim, wdt_ld) bf16, columns >= dt_rank zero
  int wdt_ld;
  int dt_rank;        // x_dbl columns >= dt_rank (the B values) are never read as dt_low
};
bool seq_dtp_supported(const ScanParams& p, const DtpArgs& q, int dtype, int dt_rank);
void seq_dtp_launch(const ScanParams& p, const DtpArgs& q, int dt_rank, hipStream_t s);
int seq_chunk_steps(int batch, int dim, int seqlen, int segments);
bool seq_dtp_chunk_supported(const ScanParams& p, const DtpArgs& q, int dtype, int segments,
                             size_t workspace_bytes);
void seq_dtp_chunk_launch(const ScanParams& p, const DtpArgs& q, int segments, void* workspace,
                          size_t workspace_bytes, void* sync, size_t sync_bytes, hipStream_t s);

}  // namespace vm
