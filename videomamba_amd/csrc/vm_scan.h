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
};


// Token-major path (vm_scan_seq.hip).  Workspace for the time-segmented form, in bytes;
// 0 when the single-pass form is chosen.  `segments` receives the chosen segment count.
// segments: 0 = cost model, > 0 forced.
size_t seq_workspace_bytes(int batch, int dim, int seqlen, int segments, int* chosen);
// Launch; `workspace` must hold seq_workspace_bytes() (or be larger).  Returns false when
// the operands do not fit the token-major kernels (the caller reports the error).
bool seq_supported(const ScanParams& p, int dtype);
void seq_launch(const ScanParams& p, int dtype, int segments, void* workspace,
                size_t workspace_bytes, hipStream_t s);

}  // namespace vm
