// KzgPcs over the eon.h device entry points (C++ mirror of kzg/src/pcs.rs:143-402 and the
// TwoAdicMultiplicativeCoset domain bookkeeping of commit/src/domain.rs).  Every matrix stays in
// HBM between stages; only commitments, opened values and witnesses come back to the host.
#pragma once
#include <stdint.h>

#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "eon.h"
#include "fr_host.h"

namespace eon_host {

// A failing eon.h call or a shape check; the C surface turns it into its code.  The reference
// panics in every one of these cases.
struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

void check(eon_ctx* ctx, int rc, const char* what);

// Owned device allocation (hipMalloc), moved not copied.
class DeviceBuffer {
  public:
    DeviceBuffer() = default;
    explicit DeviceBuffer(uint64_t bytes);
    ~DeviceBuffer();
    DeviceBuffer(DeviceBuffer&& o) noexcept : p_(o.p_), bytes_(o.bytes_) {
        o.p_ = nullptr;
        o.bytes_ = 0;
    }
    DeviceBuffer& operator=(DeviceBuffer&& o) noexcept;
    DeviceBuffer(const DeviceBuffer&) = delete;
    DeviceBuffer& operator=(const DeviceBuffer&) = delete;
    void* get() const { return p_; }
    uint64_t bytes() const { return bytes_; }
    template <class T>
    T* as() const {
        return static_cast<T*>(p_);
    }

  private:
    void* p_ = nullptr;
    uint64_t bytes_ = 0;
};

// RowMajorMatrix<Fr> on device (matrix/src/dense.rs:24-37): either owned or a view of the
// caller's buffer (the trace passed to prove).
struct DeviceMatrix {
    DeviceBuffer owned;
    const eon_fr* view = nullptr;
    uint64_t height = 0;
    uint32_t width = 0;

    const eon_fr* data() const { return view ? view : owned.as<eon_fr>(); }
    eon_fr* mutable_data() { return owned.as<eon_fr>(); }
    static DeviceMatrix alloc(uint64_t height, uint32_t width);
    static DeviceMatrix borrow(const eon_fr* p, uint64_t height, uint32_t width);
};

// TwoAdicMultiplicativeCoset: shift * <w_(2^log_size)>
struct Domain {
    Fr shift;
    uint32_t log_size;

    uint64_t size() const { return 1ull << log_size; }
    Fr generator() const { return fr_two_adic_generator(log_size); }
    Fr next_point(const Fr& x) const { return fr_mul(x, generator()); }  // domain.rs:115-117
    Domain create_disjoint_domain(uint64_t min_size) const;              // domain.rs:155-168
    std::vector<Domain> split_domains(uint32_t num_chunks) const;        // domain.rs:174-186
    bool operator==(const Domain& o) const { return shift == o.shift && log_size == o.log_size; }
};

struct PreparedDeleter {
    void operator()(eon_msm_scalars* s) const { eon_msm_scalars_destroy(s); }
};
using PreparedScalars = std::unique_ptr<eon_msm_scalars, PreparedDeleter>;

// kzg/src/pcs.rs:46-63: the committed evaluations and their coefficients, plus the coefficients'
// sorted MSM digits (kept from the commitment for the opening witnesses)
struct MatrixProverData {
    Domain domain;
    DeviceMatrix evals;
    DeviceMatrix coeffs;
    PreparedScalars prepared;
};

// one round's opened values / witnesses: [matrix][point][column]
struct Opened {
    std::vector<std::vector<std::vector<eon_fr>>> values;
    std::vector<std::vector<std::vector<eon_g1_affine>>> witnesses;
};

struct OpenRound {
    const std::vector<MatrixProverData>* data;
    std::vector<std::vector<Fr>> points;  // per matrix
};

class KzgPcs {
  public:
    KzgPcs(eon_ctx* ctx, uint64_t max_degree, const Fr& srs_alpha);
    ~KzgPcs();
    KzgPcs(const KzgPcs&) = delete;
    KzgPcs& operator=(const KzgPcs&) = delete;

    eon_ctx* ctx() const { return ctx_; }
    Domain natural_domain_for_degree(uint64_t degree) const;  // pcs.rs:218-221
    void ensure_supported(uint64_t degree) const;             // params.rs:164-173

    // pcs.rs:223-265: coset_idft_batch of each matrix, one commitment per column
    void commit(std::vector<std::pair<Domain, DeviceMatrix>> evaluations,
                std::vector<std::vector<eon_g1_affine>>& commitments, std::vector<MatrixProverData>& data);
    // commit in two halves: the coefficients of every matrix (pcs.rs:242, appended to data), then
    // the column commitments of data[first..] (pcs.rs:244-251) -- so that work which needs only
    // the coefficients (the trace LDE) can run on the auxiliary context meanwhile
    void commit_coeffs(std::vector<std::pair<Domain, DeviceMatrix>> evaluations, std::vector<MatrixProverData>& data);
    void commit_columns(std::vector<MatrixProverData>& data, size_t first,
                        std::vector<std::vector<eon_g1_affine>>& commitments);
    // pcs.rs:267-287 (values of the reference's Horner loop, from one padded coset DFT); aux:
    // on the auxiliary context (its own non-blocking stream; synchronised before returning)
    DeviceMatrix get_evaluations_on_domain(const std::vector<MatrixProverData>& data, size_t idx,
                                           const Domain& domain, bool aux = false);
    // a second context on the same device for work concurrent with this one's (null if none)
    // the auxiliary context, unless the main one is in serial mode (eon_ctx_set_serial: every
    // kernel alone on the device, for isolated profiles)
    eon_ctx* aux_live() const { return aux_ && !eon_ctx_serial(ctx_) ? aux_ : nullptr; }
    // commit/src/pcs.rs:82-101 with split_evals (domain.rs:188-221).  `only` (optional) lists the
    // chunks to commit, in order (the sharded prove gives chunk c to rank c % world); commitments
    // and data then hold those chunks only.
    void commit_quotient(const Domain& quotient_domain, const DeviceMatrix& quotient_evals, uint32_t num_chunks,
                         std::vector<std::vector<eon_g1_affine>>& commitments, std::vector<MatrixProverData>& data,
                         const std::vector<uint32_t>* only = nullptr);
    // pcs.rs:289-335: per (matrix, point) every column's value and witness.  The witness of
    // column c at z is the MSM of c's own coefficients against the opening bases H(z)
    // (eon_kzg_opening_bases_create), reusing the digits sorted at commit time, so every matrix
    // must come from commit / commit_columns (which keep those digits); otherwise EON_E_ARG.
    std::vector<Opened> open(const std::vector<OpenRound>& rounds);

  private:
    eon_ctx* ctx_;
    uint64_t max_degree_;
    eon_msm_bases* bases_ = nullptr;
    eon_ctx* aux_ = nullptr;
    void* aux_stream_ = nullptr;
};

}  // namespace eon_host
