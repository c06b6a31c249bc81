// Internal MSM API (see msm.hip; C ABI in include/eon.h).
#pragma once
#include "context.h"
#include "ec.h"

namespace eon {

// sum_i scalars[i] * bases[i] for i < n; `scalars` is a device pointer (Fr Montgomery).
Status msm_run(eon_ctx* ctx, const eon_msm_bases* bases, const Fr* scalars, uint64_t n,
               G1Affine* result);
// one MSM per column of the row-major rows x width device matrix `scalars` (result on host,
// unless out_host is null); with `keep`, the sorted digit pairs of every batch stay in it
Status msm_run_columns(eon_ctx* ctx, const eon_msm_bases* bases, const Fr* scalars, uint64_t rows,
                       uint32_t width, G1Affine* out_host, eon_msm_scalars* keep);
// out_host[t * width + j] = MSM of prepared column j against bases[t] (same window layout)
Status msm_run_prepared(eon_ctx* ctx, const eon_msm_bases* const* bases, uint32_t nbases,
                        const eon_msm_scalars* s, G1Affine* out_host);
// bases from n device (or host) affine points; force_c != 0 fixes the window size (a bases
// object whose MSMs reuse scalars prepared against another of that window size)
Status bases_create(eon_ctx* ctx, const eon_g1_affine* bases, uint64_t n, uint32_t flags,
                    bool device_ptr, eon_msm_bases** out, uint32_t force_c = 0,
                    hipStream_t stream = nullptr, DevBuf* async_tmp = nullptr);
// the bases' affine points on device, ABI form (radix-2^32 Montgomery, (0,0) = identity)
const G1Affine* bases_points(const eon_msm_bases* b);
uint32_t bases_window(const eon_msm_bases* b);
bool bases_precomputed(const eon_msm_bases* b);
// release a bases object (caller holds ctx->mu and has synchronised its work)
void bases_free(eon_msm_bases* b);
// the window table in 29-Montgomery form (precomputed radix-2^29 bases; else null), its windows
const G1Affine* bases_table29(const eon_msm_bases* b);
// 3 x that table (same layout, 29-form), built on the first call (synchronises `st` then); null
// when the bases have no radix-2^29 table or the allocation fails
const G1Affine* bases_table3_29(const eon_msm_bases* b, hipStream_t st);
uint32_t bases_windows(const eon_msm_bases* b);
// fixed-base bases whose window table the caller writes (affine, radix-2^32 ABI form, entry
// i * windows + w = 2^(c w) P_i), then seals: points <- the w = 0 entries, table -> 29-form
Status bases_alloc_table(eon_ctx* ctx, uint64_t n, uint32_t c, eon_msm_bases** out);
G1Affine* bases_table_mut(eon_msm_bases* b);
Status bases_seal_table(eon_msm_bases* b, hipStream_t st);

// XYZZ -> affine on the host (Montgomery batch inversion, 64-bit limbs; the same bytes as the
// device conversion)
void host_xyzz_to_affine(const G1Xyzz* in, uint64_t m, G1Affine* out);

constexpr uint32_t BATCH = 32;  // points per thread in batched XYZZ -> affine conversion
hipError_t launch_batch_to_affine(const G1Xyzz* in, uint64_t m, G1Affine* out, hipStream_t st);

}  // namespace eon
