/*
 * eon.h -- C ABI of the MI355X (gfx950) prover hot path for the plonky3-eon BN254/KZG stack.
 *
 * This is the drop-in boundary: every entry point replaces one reference interface on the
 * prover path, cited below as reference file:line (reference = Lolazyx/plonky3-eon).  Plain
 * pointers and sizes only; no torch or HIP types in signatures (streams are passed as void*).
 * A Rust shim binds these with `extern "C"`.
 *
 * Data layout (shared with the reference, zero-copy):
 *   eon_fr        = p3_bn254::Fr: [u64;4] little-endian Montgomery residue a*2^256 mod r,
 *                   canonical (< r)                                   (bn254/src/field.rs:98-105)
 *   matrices      = p3_matrix RowMajorMatrix<Fr>: element (row, col) at values[row*width + col]
 *                                                                     (matrix/src/dense.rs:24-37)
 *   eon_g1_affine = BN254 G1 affine point, x and y as Fq Montgomery residues (R = 2^256 mod q),
 *                   [u64;4] LE each; the point at infinity is encoded as x = y = 0.
 *
 * Conventions:
 *   - return 0 on success, a negative EON_E_* code otherwise; eon_last_error() has the message.
 *     The reference panics in these cases (assert!/log2_strict_usize/unwrap); a Rust shim
 *     should panic on a nonzero return to keep that behaviour.
 *   - `*_dev` entry points take DEVICE pointers and enqueue asynchronously on the context's
 *     stream (eon_ctx_set_stream); the others take HOST pointers and are synchronous.
 *   - a context is internally locked: entry points are thread-safe (the reference's DFTs are
 *     Clone + Sync and share twiddle caches, dft/src/radix_2_dit_parallel.rs:30-40).
 */
#ifndef EON_H
#define EON_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    uint64_t l[4];
} eon_fr;

typedef struct {
    uint64_t x[4];
    uint64_t y[4];
} eon_g1_affine;

/* BN254 G2 affine point on the sextic twist over Fq2 = Fq[u]/(u^2 + 1): x = x[0] + x[1] u (Fq
 * Montgomery [u64;4] LE each), identity = all zero.  Gt / Fq12 element in the tower
 * Fq12 = Fq6[w]/(w^2 - v), Fq6 = Fq2[v]/(v^3 - (9 + u)): c[2k], c[2k+1] = the Fq2 coefficient k
 * in the order c0.c0, c0.c1, c0.c2, c1.c0, c1.c1, c1.c2 (halo2curves' Fq12 layout). */
typedef struct {
    uint64_t x[2][4];
    uint64_t y[2][4];
} eon_g2_affine;

typedef struct {
    uint64_t c[12][4];
} eon_fq12;

typedef struct eon_ctx eon_ctx;

/* Collectives over DEVICE buffers among `world` processes (one per GPU), called with a context's
 * stream; each must leave recv complete and ordered before that stream's later work (an RCCL call
 * enqueued on `hip_stream` does; a host-staged one synchronizes).
 *   all_gather: recv receives `world` blocks of `bytes`, in rank order.  Used by the lane-sharded
 *               prove (eon_prove.h), a context's sharded work (eon_ctx_set_collective) and
 *               eon_msm_sharded_dev.
 *   all_to_all: send holds `world` blocks of `bytes` (block h goes to rank h); recv receives
 *               `world` blocks, block g from rank g (ncclAllToAll).  Used by
 *               eon_fourstep_dft_dev; may be NULL when no four-step transform runs. */
typedef struct {
    uint32_t rank;
    uint32_t world;
    int (*all_gather)(void* user, const void* send, void* recv, uint64_t bytes, void* hip_stream);
    void* user;
    int (*all_to_all)(void* user, const void* send, void* recv, uint64_t bytes, void* hip_stream);
} eon_collective;
typedef struct eon_msm_bases eon_msm_bases;
typedef struct eon_msm_scalars eon_msm_scalars;

enum {
    EON_OK = 0,
    EON_E_SHAPE = -1,            /* height not a power of two, size mismatch (reference: panic) */
    EON_E_DEGREE_TOO_LARGE = -2, /* KzgError::DegreeTooLarge (kzg/src/params.rs:164-173) */
    EON_E_DEVICE = -3,           /* HIP runtime error */
    EON_E_OOM = -4,              /* device allocation failed */
    EON_E_ARG = -5               /* null pointer / invalid argument */
};

enum {
    EON_ORDER_NATURAL = 0, /* RowMajorMatrix output, as Radix2Dit (dft/src/radix_2_dit.rs:61-77) */
    EON_ORDER_BITREV = 1   /* storage of Radix2DitParallel's BitReversedMatrixView: storage row
                              reverse_bits_len(k, log2 h) holds logical row k
                              (dft/src/radix_2_dit_parallel.rs:146,165,227) */
};

/* output layouts of eon_fourstep_dft_dev */
enum {
    EON_FOURSTEP_NATURAL = 0,    /* rank g holds X[g N/G, (g+1) N/G): its contiguous natural slice
                                    (a second all_to_all) */
    EON_FOURSTEP_TRANSPOSED = 1  /* rank g holds the N2 x N1/G row-major block of the N2 x N1 view:
                                    row k2, column k1' = X[N1 k2 + g N1/G + k1'] (one all_to_all) */
};

/* ---- context ---------------------------------------------------------------------------- */
int eon_ctx_create(int device_ordinal, eon_ctx** out);
void eon_ctx_destroy(eon_ctx* ctx);
const char* eon_last_error(const eon_ctx* ctx);
/* Stream (a hipStream_t) for all subsequent work of this context, used verbatim: NULL selects
 * the HIP null (default) stream.  Until the first call the context uses a stream of its own. */
int eon_ctx_set_stream(eon_ctx* ctx, void* hip_stream);
/* The stream the context currently enqueues on (as set, or its own). */
void* eon_ctx_stream(eon_ctx* ctx);
/* The device ordinal the context was created on. */
int eon_ctx_device(const eon_ctx* ctx);
/* Bind the context to a process group (copied; NULL or world <= 1 unbinds).  Work that is the
 * same on every rank then splits across the ranks: eon_kzg_opening_bases_create(_many) computes
 * 1/world of the rows and all-gathers the tables.  Every rank must then make the same calls in
 * the same order. */
int eon_ctx_set_collective(eon_ctx* ctx, const eon_collective* coll);
int eon_ctx_synchronize(eon_ctx* ctx);
/* Give back to the device every cached idle buffer of the context: the transient-buffer pool
 * (KZG opening-bases tables and scratch; capped at EON_POOL_CAP_GB, default 8, read at creation)
 * and the kept sorted-digit buffers of destroyed eon_msm_scalars (capped at 48 GB).  Synchronizes
 * the context's streams first.  Call it between proofs when another allocator in the process
 * (e.g. torch's caching allocator) needs the memory; the next proof allocates afresh. */
int eon_ctx_trim(eon_ctx* ctx);
/* Per-launch kernel timing with HIP events on the launch stream (the analogue of the
 * reference's tracing spans, e.g. dft/src/radix_2_dit_parallel.rs:168).  eon_ctx_profile(ctx, 1)
 * clears the record and starts recording; eon_ctx_profile_report writes a JSON object
 * {kernel: {launches, total_ms, alg_bytes}} into buf (synchronizes on the recorded events). */
int eon_ctx_profile(eon_ctx* ctx, int enable);
int eon_ctx_profile_report(eon_ctx* ctx, char* buf, uint64_t len);
/* Serial mode (also EON_SERIAL=1 at creation): every kernel of this context on its one stream,
 * none on the MSM / opening side streams, so that each launch runs alone on the device and its
 * event-timed or profiler duration is isolated.  For measurement only: results are identical,
 * the prove is slower (no overlap of digit sorts with piece sums). */
int eon_ctx_set_serial(eon_ctx* ctx, int serial);
int eon_ctx_serial(const eon_ctx* ctx);
/* ---- diagnostics (measurement only; not on any product path) ------------------------------ */
typedef struct {
    double clock_mhz_median; /* in-kernel shader clock: delta s_memtime / delta s_memrealtime x 100 MHz */
    double clock_mhz_min;    /* over the blocks of the last launch */
    double clock_mhz_max;
    double products_per_s;   /* radix-2^29 Montgomery products per second over the timed launches */
    double ms_per_launch;
} eon_clock_probe;
/* Run `launches` back-to-back launches of a radix-2^29 product chain (`iters` products per chain,
 * two chains per thread, 4096 x 256 threads) on the context stream, after one untimed launch, and
 * report the shader clock the chip held (median over blocks of the last launch) and the product
 * rate (MI355X_MICROARCH.md, DVFS item 6).  Synchronous. */
int eon_diag_clock_probe(eon_ctx* ctx, uint32_t launches, uint32_t iters, eon_clock_probe* out);
/* Self-check of the whole-product asm statements the MSM piece sums use (prod_asm.h) against the
 * column-block products, bit for bit, on n pseudo-random operands of each kind at their limb
 * bounds (half of them at the maximum limb); mismatches[0..2] = mismatching mul / sqr / sum2
 * cases. */
int eon_diag_prod_asm_check(eon_ctx* ctx, uint32_t n, uint32_t seed, uint32_t mismatches[3]);

/* ABI version; bumped on any signature or struct-layout change (4: the verifier pairings and their
 * eon_g2_affine / eon_fq12 types; 3: eon_collective's all_to_all field).  Bindings must check it
 * at load time: a binding built against an older layout would pass a shorter eon_collective. */
uint32_t eon_abi_version(void);

/* ---- TwoAdicSubgroupDft<Fr> (dft/src/traits.rs:27-249) -----------------------------------
 * `in` is height x width, row-major.  height must be a power of two with log2(height) (+ added
 * bits) <= 28 (Fr::TWO_ADICITY, bn254/src/field.rs:564).  `in` and `out` may alias. */

/* dft_batch (dft/src/traits.rs:61): coefficients -> evaluations on H. */
int eon_dft_batch(eon_ctx* ctx, const eon_fr* in, eon_fr* out, uint64_t height, uint32_t width,
                  int out_order);
/* idft_batch (dft/src/traits.rs:111-122): evaluations on H -> coefficients (natural order). */
int eon_idft_batch(eon_ctx* ctx, const eon_fr* in, eon_fr* out, uint64_t height, uint32_t width);
/* coset_dft_batch (dft/src/traits.rs:83-91): coefficients -> evaluations on shift*H. */
int eon_coset_dft_batch(eon_ctx* ctx, const eon_fr* in, eon_fr* out, uint64_t height,
                        uint32_t width, const eon_fr* shift, int out_order);
/* coset_idft_batch (dft/src/traits.rs:144-153): evaluations on shift*H -> coefficients. */
int eon_coset_idft_batch(eon_ctx* ctx, const eon_fr* in, eon_fr* out, uint64_t height,
                         uint32_t width, const eon_fr* shift);
/* coset_lde_batch (dft/src/traits.rs:226-249; Radix2DitParallel override at
 * dft/src/radix_2_dit_parallel.rs:169-228): evaluations on H -> evaluations on shift*K,
 * |K| = height << added_bits.  `out` holds (height << added_bits) x width.  shift NULL = ONE
 * (lde_batch, dft/src/traits.rs:187-192).  `shift` is always a host pointer. */
int eon_coset_lde_batch(eon_ctx* ctx, const eon_fr* in, eon_fr* out, uint64_t height,
                        uint32_t width, uint32_t added_bits, const eon_fr* shift, int out_order);
/* coset_dft_batch of the COEFFICIENT matrix zero-padded to height << added_bits -- the second
 * half of coset_lde_batch (dft/src/traits.rs:226-249), and KzgPcs::get_evaluations_on_domain from
 * the committed coefficients (kzg/src/pcs.rs:267-287, commit/src/testing.rs:93-105):
 * out[k] = sum_j coeffs[j] (shift * w^k)^j, |K| = height << added_bits.  `in` != `out`. */
int eon_coset_dft_padded_batch(eon_ctx* ctx, const eon_fr* coeffs, eon_fr* out, uint64_t height,
                               uint32_t width, uint32_t added_bits, const eon_fr* shift,
                               int out_order);

/* device-pointer variants (same semantics, asynchronous on the context stream) */
int eon_dft_batch_dev(eon_ctx* ctx, const eon_fr* in, eon_fr* out, uint64_t height,
                      uint32_t width, int out_order);
int eon_idft_batch_dev(eon_ctx* ctx, const eon_fr* in, eon_fr* out, uint64_t height,
                       uint32_t width);
int eon_coset_dft_batch_dev(eon_ctx* ctx, const eon_fr* in, eon_fr* out, uint64_t height,
                            uint32_t width, const eon_fr* shift, int out_order);
int eon_coset_idft_batch_dev(eon_ctx* ctx, const eon_fr* in, eon_fr* out, uint64_t height,
                             uint32_t width, const eon_fr* shift);
int eon_coset_lde_batch_dev(eon_ctx* ctx, const eon_fr* in, eon_fr* out, uint64_t height,
                            uint32_t width, uint32_t added_bits, const eon_fr* shift,
                            int out_order);
int eon_coset_dft_padded_batch_dev(eon_ctx* ctx, const eon_fr* coeffs, eon_fr* out, uint64_t height,
                                   uint32_t width, uint32_t added_bits, const eon_fr* shift,
                                   int out_order);

/* ---- BN254 G1 multi-scalar multiplication -------------------------------------------------
 * Value of G1::multi_exp (bn254/src/curve.rs:158-179, halo2curves msm_best): sum_i s_i * P_i,
 * returned in affine form ((0,0) = identity; empty input -> identity).  Bases are uploaded
 * once into an eon_msm_bases handle and reused, as the KZG SRS g1_powers is
 * (kzg/src/params.rs:57-139, commit_column kzg/src/util.rs:37-40). */
enum {
    EON_MSM_PRECOMPUTE = 1 /* fixed-base mode: store 2^(c*w) * P_i for every window (SRS bases) */
};
/* `bases`: host array of n affine points with canonical coordinates. */
int eon_msm_bases_create(eon_ctx* ctx, const eon_g1_affine* bases, uint64_t n, uint32_t flags,
                         eon_msm_bases** out);
void eon_msm_bases_destroy(eon_msm_bases* bases);
uint64_t eon_msm_bases_len(const eon_msm_bases* bases);
/* MSM over the first n bases; `scalars` host (eon_msm_g1) or device (eon_msm_g1_dev) Fr array;
 * `out` is a host pointer; both calls return when the result is in *out.  n > len(bases) is
 * EON_E_SHAPE (the reference asserts equal lengths, curve.rs:159-162). */
int eon_msm_g1(eon_ctx* ctx, const eon_msm_bases* bases, const eon_fr* scalars, uint64_t n,
               eon_g1_affine* out);
int eon_msm_g1_dev(eon_ctx* ctx, const eon_msm_bases* bases, const eon_fr* scalars, uint64_t n,
                   eon_g1_affine* out);
/* One MSM per column of a row-major rows x width Fr matrix over bases[0..rows): out[j] =
 * sum_i mat[i][j] * P_i (width affine points, host) -- the per-column commit_column loop of
 * KzgPcs::commit (kzg/src/pcs.rs:244-251) and of open's witnesses (pcs.rs:310-316).  `mat` is
 * host (eon_msm_g1_columns) or device (eon_msm_g1_columns_dev). */
int eon_msm_g1_columns(eon_ctx* ctx, const eon_msm_bases* bases, const eon_fr* mat, uint64_t rows,
                       uint32_t width, eon_g1_affine* out);
int eon_msm_g1_columns_dev(eon_ctx* ctx, const eon_msm_bases* bases, const eon_fr* mat,
                           uint64_t rows, uint32_t width, eon_g1_affine* out);
/* quotient_and_eval (kzg/src/util.rs:100-111) for every column of a row-major rows x width
 * coefficient matrix (device) at `point` (host): quotient (device) receives the (rows-1) x width
 * synthetic-division quotients, values (device) the width evaluations f_j(point), as
 * KzgPcs::open computes per (matrix, point, column) (kzg/src/pcs.rs:297-330).  quotient NULL:
 * values only. */
int eon_quotient_and_eval_columns_dev(eon_ctx* ctx, const eon_fr* coeffs, uint64_t rows,
                                      uint32_t width, const eon_fr* point, eon_fr* quotient,
                                      eon_fr* values);
/* The remainder of quotient_and_eval (kzg/src/util.rs:100-111) only -- f_j(z) for every column
 * of the rows x width coefficient matrix (device) at npoints points (host array): values
 * (device) receives npoints x width Fr, values[t * width + j] = f_j(points[t]).  One read of the
 * coefficients serves up to four points (KzgPcs::open's opened values, kzg/src/pcs.rs:305-316). */
int eon_eval_columns_dev(eon_ctx* ctx, const eon_fr* coeffs, uint64_t rows, uint32_t width,
                         const eon_fr* points, uint32_t npoints, eon_fr* values);
/* As eon_msm_bases_create with `bases` a DEVICE pointer (coordinates are not re-validated). */
int eon_msm_bases_create_dev(eon_ctx* ctx, const eon_g1_affine* bases, uint64_t n, uint32_t flags,
                             eon_msm_bases** out);
/* One-shot G1::multi_exp(points, scalars) on host arrays (bases uploaded for this call only). */
int eon_g1_multi_exp(eon_ctx* ctx, const eon_g1_affine* points, const eon_fr* scalars, uint64_t n,
                     eon_g1_affine* out);

/* Prepared scalar columns.  eon_msm_g1_columns_prepare_dev is eon_msm_g1_columns_dev (out may be
 * NULL) that also keeps every column's sorted bucket digits on device in *prepared
 * (~8 bytes x rows x ceil(255/c) per column), so that MSMs of the SAME columns against other
 * bases of the same window layout skip the digit extraction and sort:
 * eon_msm_g1_columns_prepared writes out[t * width + j] = sum_i mat[i][j] * bases[t][i].  KzgPcs
 * commits a matrix with the first (kzg/src/pcs.rs:244-251) and opens it with the second against
 * eon_kzg_opening_bases_create bases (pcs.rs:305-316).  `mat` need not outlive the prepare call;
 * every bases[t] must hold >= rows points with the window layout of the prepare call's bases
 * (EON_E_SHAPE otherwise). */
int eon_msm_g1_columns_prepare_dev(eon_ctx* ctx, const eon_msm_bases* bases, const eon_fr* mat,
                                   uint64_t rows, uint32_t width, eon_g1_affine* out,
                                   eon_msm_scalars** prepared);
int eon_msm_g1_columns_prepared(eon_ctx* ctx, const eon_msm_bases* const* bases, uint32_t nbases,
                                const eon_msm_scalars* prepared, eon_g1_affine* out);
void eon_msm_scalars_destroy(eon_msm_scalars* prepared);
/* KZG opening bases for `point` z (host) over the first n-1 points G_i of `srs`:
 * H_j = sum_{i<j} z^(j-1-i) G_i, j < n (H_0 = identity), in the window layout of `srs`.  For any
 * coefficient column c of length n, sum_j c_j H_j = commit_column(quotient_and_eval(c, z).0)
 * (kzg/src/util.rs:37-40,100-111): the opening witness of KzgPcs::open (kzg/src/pcs.rs:305-316)
 * as an MSM of the committed coefficients themselves. */
int eon_kzg_opening_bases_create(eon_ctx* ctx, const eon_msm_bases* srs, uint64_t n,
                                 const eon_fr* point, eon_msm_bases** out);
/* The same for npoints points (host array) at once (the points' constructions overlap on the
 * device): outs[t] = the opening bases of points[t]. */
int eon_kzg_opening_bases_create_many(eon_ctx* ctx, const eon_msm_bases* srs, uint64_t n,
                                      const eon_fr* points, uint32_t npoints, eon_msm_bases** outs);

/* ---- eon-uni-stark quotient on the Poseidon2-AIR --------------------------------------------
 * selectors_on_coset (commit/src/domain.rs:252-292): for the trace domain H (shift 1, 2^log_n) on
 * the coset shift * K (2^log_q), writes 4 x 2^log_q Fr to device `out`: is_first_row,
 * is_last_row, is_transition, inv_vanishing.  shift (host) must not be ONE (domain.rs:254). */
int eon_selectors_on_coset_dev(eon_ctx* ctx, uint32_t log_n, uint32_t log_q, const eon_fr* shift,
                               eon_fr* out);

/* Poseidon2-AIR over BN254 Fr (poseidon2-air/src/air.rs): WIDTH 3, SBOX_DEGREE 5,
 * SBOX_REGISTERS 1, external layer mds_light, internal layer [2,1,1;1,2,1;1,1,3]
 * (bn254/src/poseidon2.rs:55-63); VECTOR_LEN permutations per row (vectorized.rs).  Constants
 * are host arrays: beginning/ending half_full_rounds x 3, partial partial_rounds
 * (RoundConstants, poseidon2-air/src/constants.rs:17-31). */
typedef struct {
    uint32_t half_full_rounds;
    uint32_t partial_rounds;
    const eon_fr* beginning;
    const eon_fr* partial;
    const eon_fr* ending;
} eon_poseidon2_constants;
typedef struct eon_p2air eon_p2air;
/* Poseidon2Air::new / VectorizedPoseidon2Air::new (vector_len: power of two <= 32) */
int eon_p2air_create(eon_ctx* ctx, const eon_poseidon2_constants* constants, uint32_t vector_len,
                     eon_p2air** out);
void eon_p2air_destroy(eon_p2air* air);
/* trace width: (4 + 12 * half_full_rounds + 2 * partial_rounds) * vector_len (164 * vector_len) */
uint32_t eon_p2air_width(const eon_p2air* air);
/* VECTOR_LEN, and the constraints of one permutation: 12 * half_full_rounds + 2 * partial_rounds
 * (160; the folder's per-lane block, eon-uni-stark/src/folder.rs:81-85) */
uint32_t eon_p2air_vector_len(const eon_p2air* air);
uint32_t eon_p2air_constraints_per_perm(const eon_p2air* air);
/* generate_vectorized_trace_rows (poseidon2-air/src/generation.rs:14-72): inputs n_perms x 3 Fr
 * (device), trace (n_perms / vector_len) x width (device); n_perms = vector_len * 2^k. */
int eon_p2air_generate_trace_dev(eon_ctx* ctx, const eon_p2air* air, const eon_fr* inputs,
                                 uint64_t n_perms, eon_fr* trace);
/* quotient_values (eon-uni-stark/src/prover.rs:539-709) with the ProverConstraintFolder
 * accumulator (folder.rs:81-85): `lde` is the trace on the quotient domain GENERATOR * K,
 * |K| = 2^(log_n + log_qd), natural order (KzgPcs::get_evaluations_on_domain), device;
 * out[i] = sum_k alpha^(K-1-k) C_k(row i) * inv_vanishing[i], device, 2^(log_n+log_qd) Fr.
 * `alpha` is a host pointer. */
int eon_p2air_quotient_values_dev(eon_ctx* ctx, const eon_p2air* air, const eon_fr* lde,
                                  uint32_t log_n, uint32_t log_qd, const eon_fr* alpha,
                                  eon_fr* out);

/* ---- generic AIR: quotient_values for any EonAir ---------------------------------------------
 * The constraints get_symbolic_constraints returns (eon-uni-stark/src/symbolic_builder.rs:72-126)
 * as a DAG of SymbolicExpression nodes (symbolic_expression.rs:78-145; SymbolicVariable /
 * Entry, symbolic_variable.rs:8-40), in topological order: every operand index is smaller than
 * its user's (a shared Arc is emitted once and referenced by index).  `constraints` lists the
 * root node of each constraint in assert order (the folder's constraint_index order,
 * folder.rs:81-85).  Leaves: EON_SYM_CONSTANT a = index into consts (canonical Fr);
 * EON_SYM_MAIN a = column, b = row offset (0 local, 1 next); EON_SYM_PUBLIC a = public index;
 * the three selectors (symbolic_builder.rs:205-221).  Preprocessed, permutation (LogUp) and
 * challenge variables are rejected (EON_E_ARG): the prove path has no preprocessed data and no
 * lookups (prover.rs:211-250 None branch). */
enum {
    EON_SYM_CONSTANT = 0,
    EON_SYM_MAIN = 1,
    EON_SYM_PUBLIC = 2,
    EON_SYM_IS_FIRST_ROW = 3,
    EON_SYM_IS_LAST_ROW = 4,
    EON_SYM_IS_TRANSITION = 5,
    EON_SYM_ADD = 6, /* a + b */
    EON_SYM_SUB = 7, /* a - b */
    EON_SYM_NEG = 8, /* -a */
    EON_SYM_MUL = 9, /* a * b */
    EON_SYM_PREPROCESSED = 10,
    EON_SYM_PERMUTATION = 11,
    EON_SYM_CHALLENGE = 12
};
typedef struct {
    uint32_t kind;
    uint32_t a;
    uint32_t b;
} eon_sym_node;
typedef struct eon_air_program eon_air_program;
typedef struct {
    uint32_t width;                 /* main trace width */
    uint32_t num_public_values;
    uint32_t num_constraints;
    uint32_t max_constraint_degree; /* get_max_constraint_degree (symbolic_builder.rs:46-69) */
    uint32_t num_instructions;      /* compiled program (after common-subexpression elimination) */
    uint32_t num_registers;
    uint32_t num_constants;
} eon_air_program_stats;
/* Compile the constraint DAG for a trace of `width` columns and n_public public values. */
int eon_air_program_create(eon_ctx* ctx, const eon_sym_node* nodes, uint32_t n_nodes, const eon_fr* consts,
                           uint32_t n_consts, const uint32_t* constraints, uint32_t n_constraints,
                           uint32_t width, uint32_t n_public, eon_air_program** out);
void eon_air_program_destroy(eon_air_program* prog);
int eon_air_program_info(const eon_air_program* prog, eon_air_program_stats* out);
/* get_log_quotient_degree (symbolic_builder.rs:15-43): log2_ceil(max(max_degree + is_zk, 2) - 1) */
uint32_t eon_air_program_log_quotient_degree(const eon_air_program* prog, uint32_t is_zk);
/* quotient_values (eon-uni-stark/src/prover.rs:539-709) of the program: `lde` = the trace on the
 * quotient domain GENERATOR * K, |K| = 2^(log_n + log_qd), natural order, device, width columns;
 * publics = host array of n_public Fr (public_values); alpha host.  out (device, 2^(log_n+log_qd)
 * Fr) = sum_k alpha^(K-1-k) C_k(local = row i, next = row (i + 2^log_qd) mod Q, selectors of
 * selectors_on_coset, publics) * inv_vanishing[i]. */
int eon_quotient_values_dev(eon_ctx* ctx, const eon_air_program* prog, const eon_fr* lde, uint32_t log_n,
                            uint32_t log_qd, const eon_fr* alpha, const eon_fr* publics, uint32_t n_public,
                            eon_fr* out);

/* out[i] = sum_{j<k} coeffs[j] * in[j * rows + i] (device in/out, host coeffs, 1 <= k <= 64):
 * the combine step of the lane-sharded quotient -- every rank all-gathers the
 * shards' partial quotients and weights shard g by alpha^(K_lane * (VECTOR_LEN - lane_end_g)). */
int eon_fr_lincomb_dev(eon_ctx* ctx, const eon_fr* in, uint32_t k, uint64_t rows,
                       const eon_fr* coeffs, eon_fr* out);

/* ---- four-step NTT across ranks (BASELINE configs[4]) ------------------------
 * Step 2 + the local half of step 3 of a size-2^log_n forward DFT split as N1 x N2
 * (N1 = 2^log_n1): y is the rank's N1 x cols block (columns col0 .. col0+cols of the N1 x N2 view
 * x[N2 i1 + i2], after a size-N1 eon_dft_batch_dev over its columns); writes
 * send[h][i2][k1'] = y[h N1/parts + k1'][i2] * w_N^((col0 + i2)(h N1/parts + k1')), i.e. `parts`
 * contiguous cols x (N1/parts) blocks, one per destination rank (device pointers). */
int eon_fourstep_twiddle_pack_dev(eon_ctx* ctx, const eon_fr* y, uint32_t log_n, uint32_t log_n1,
                                  uint64_t col0, uint32_t cols, uint32_t parts, eon_fr* send);

/* The whole sharded forward DFT: dft_batch (dft/src/traits.rs:61, natural order; the reference
 * has no multi-GPU path -- this is SURVEY.md 8(e)'s four-step scheme) of ONE column of N = 2^log_n
 * elements spread over the collective's `world` ranks (every rank calls with the same log_n,
 * layout and collective; world must divide N2 and N1, N1 = 2^ceil(log_n / 2), N2 = N / N1).
 *   in:  the rank's N1 x (N2/world) row-major block of the N1 x N2 view x[N2 i1 + i2]: columns
 *        [rank N2/world, (rank+1) N2/world) -- i.e. in[i1 C + c] = x[N2 i1 + rank C + c];
 *   out: N/world elements in `layout` (EON_FOURSTEP_NATURAL or EON_FOURSTEP_TRANSPOSED).
 * Steps: size-N1 column DFTs, twiddles w_N^(i2 k1) fused with the pack per destination,
 * all_to_all, size-N2 DFTs, and for the natural layout a second all_to_all plus a block
 * interleave.  coll NULL = the context's bound collective (eon_ctx_set_collective), or one rank.
 * Device pointers; `in` is not modified.  Synchronous with respect to the collective calls. */
int eon_fourstep_dft_dev(eon_ctx* ctx, const eon_fr* in, eon_fr* out, uint32_t log_n, int layout,
                         const eon_collective* coll);

/* G1::multi_exp (bn254/src/curve.rs:158-179) of ONE MSM whose terms are split over the ranks by
 * contiguous range (SURVEY.md 8(e), configs[4] (ii)): every rank passes its bases (over its own
 * range) and its n_local scalars (device pointer); each runs a full Pippenger, the `world` affine
 * partial points are all-gathered (64 B per rank) and summed (EC additions -- not an RCCL
 * reduction).  Every rank receives the same result in *out (host).  coll NULL = the context's
 * bound collective, or one rank. */
int eon_msm_sharded_dev(eon_ctx* ctx, const eon_msm_bases* bases, const eon_fr* scalars, uint64_t n_local,
                        const eon_collective* coll, eon_g1_affine* out);

/* ---- test SRS (setup, not prove time) --------------------------------------------------------
 * init_srs_unsafe's g1_powers (kzg/src/params.rs:123-139): out[i] = alpha^i * G1::generator(),
 * affine, i < n.  `alpha` is a host pointer; `out` host (eon_g1_srs_powers) or device (_dev). */
int eon_g1_srs_powers(eon_ctx* ctx, const eon_fr* alpha, uint64_t n, eon_g1_affine* out);
int eon_g1_srs_powers_dev(eon_ctx* ctx, const eon_fr* alpha, uint64_t n, eon_g1_affine* out);

/* ---- verifier pairings (setup / verify, not prove time) --------------------
 * All host pointers, synchronous.  G1 / G2 inputs must be canonical and on their curves
 * (EON_E_ARG otherwise).
 *
 * eon_g2_mul: out = k * base (base NULL = G2::generator()); init_srs_unsafe's
 *   g2_alpha = [alpha] G2 (kzg/src/params.rs:123-139), G2::mul_scalar (bn254/src/curve.rs).
 * eon_multi_pairing: out = prod_i e(p[i], q[i]) (multi_pairing, bn254/src/curve.rs:439-452;
 *   pairing, :429-436, is n = 1): the optimal-ate Miller loops and one final exponentiation; the
 *   identity of Gt (Fq12 one) for n = 0.
 * eon_kzg_verify_batch: *ok = 1 iff prod_i e(C_i - v_i G1, G2) e(-W_i, g2_alpha - z_i G2) is the
 *   identity -- verify_batch (kzg/src/util.rs:245-292; for n = 1 verify_single, :150-168, whose
 *   e(C - vG1, G2) == e(W, g2_alpha - zG2) is the same condition).  *ok = 0 is the reference's
 *   Err(KzgError::ProofShapeMismatch); n = 0 is Ok.  Pairs sharing a G2 argument are merged by
 *   bilinearity before the Miller loops (one pairing per distinct opening point, plus one). */
int eon_g2_mul(eon_ctx* ctx, const eon_g2_affine* base, const eon_fr* k, eon_g2_affine* out);
int eon_multi_pairing(eon_ctx* ctx, const eon_g1_affine* p, const eon_g2_affine* q, uint64_t n, eon_fq12* out);
int eon_kzg_verify_batch(eon_ctx* ctx, const eon_g1_affine* commitments, const eon_g1_affine* witnesses,
                         const eon_fr* values, const eon_fr* points, uint64_t n, const eon_g2_affine* g2_alpha,
                         int* ok);

#ifdef __cplusplus
}
#endif
#endif /* EON_H */
