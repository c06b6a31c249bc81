// Internal MSM API (see msm.hip; C ABI in include/eon.h).
#pragma once
#include "context.h"
#include "ec.h"

namespace eon {

// sum_i scalars[i] * bases[i] for i < n; `scalars` is a device pointer (Fr Montgomery).
Status msm_run(eon_ctx* ctx, const eon_msm_bases* bases, const Fr* scalars, uint64_t n,
               G1Affine* result);
// one MSM per column of the row-major rows x width device matrix `scalars` (result on host)
Status msm_run_columns(eon_ctx* ctx, const eon_msm_bases* bases, const Fr* scalars, uint64_t rows,
                       uint32_t width, G1Affine* out_host);

constexpr uint32_t BATCH = 32;  // points per thread in batched XYZZ -> affine conversion
hipError_t launch_batch_to_affine(const G1Xyzz* in, uint64_t m, G1Affine* out, hipStream_t st);

}  // namespace eon
