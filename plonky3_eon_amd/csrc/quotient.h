// Shared by quotient.hip (Poseidon2-AIR fused kernel) and air_program.hip (generic AIRs).
#pragma once
#include "context.h"

namespace eon {

// log_q - log_n <= 16, log_q <= 28
Status check_domains(uint32_t log_n, uint32_t log_q);
// Z_H(x_i) = shift^n w_rate^j - 1 and its inverse for the 2^(log_q - log_n) distinct values
// (ctx->sel_tab); enqueued on ctx->stream
Status vanishing_table(eon_ctx* ctx, uint32_t log_n, uint32_t log_q, const Fr& shift, Fr** zh, Fr** zh_inv);
// selectors_on_coset (commit/src/domain.rs:252-292) into out[0..4q): is_first_row, is_last_row,
// is_transition, inv_vanishing; shift != 1; enqueued on ctx->stream
Status selectors_launch(eon_ctx* ctx, uint32_t log_n, uint32_t log_q, const Fr& shift, Fr* out);

}  // namespace eon
