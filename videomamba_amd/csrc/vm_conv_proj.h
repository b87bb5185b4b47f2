// Shared declarations of the token-major mixer-middle kernels (vm_conv_proj.hip: one
// workgroup per 64 token rows, all channels; vm_conv_proj_sk.hip: the split-K form used
// for small batches).
#pragma once

#include "vm_common.h"

namespace vm {

// Raw arguments of vm_conv_proj_fwd (token-major rows: element (token, channel) at
// base + token * *_tl + channel; tokens are batch-contiguous, token = b * out_len + t).
struct ConvProjTmArgs {
  const bf16_t* x; long long x_tl;
  const float* cw; const float* cb;
  const void* csi; int csi_dtype; long long csi_sb, csi_sd;
  void* cso; int cso_dtype; long long cso_sb, cso_sd;  // new conv state (nullable)
  const bf16_t* wx; int e, e_pad;
  const bf16_t* wdt; int r, r_pad;   // wdt == nullptr: no dt_proj
  bf16_t* u; long long u_tl;
  bf16_t* xdbl; long long xd_tl;
  bf16_t* dt; long long dt_tl;
  int out_len, batch, dim, seqlen, width;
};

// The split-K form runs for batch <= kSkMaxBatch.  The choice depends on the batch only,
// never on the sequence length, so a sequence run in chunks sees the same arithmetic as
// the full-sequence run (chunked == full bitwise).
constexpr int kSkMaxBatch = 8;
constexpr int kSkMaxEp = 76;  // round_up(R + 2N, 4) the split-K form stages per token row
long long conv_proj_sk_workspace_bytes(int batch, int out_len, int dim, int e);
void conv_proj_sk_launch(const ConvProjTmArgs& a, float* part, hipStream_t s);
// its second kernel alone (partials -> x_dbl [-> dt]), shared with vm_inproj_conv.hip
void conv_proj_sk_reduce_launch(const ConvProjTmArgs& a, float* part, hipStream_t s);
// The fused small-batch form (one launch, no partials; bit-identical to the split-K form)
// for dim <= 1152 and out_len >= 16.
bool conv_proj_fused_ok(const ConvProjTmArgs& a);
void conv_proj_fused_launch(const ConvProjTmArgs& a, hipStream_t s);

}  // namespace vm
