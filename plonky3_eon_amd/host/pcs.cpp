// KzgPcs over eon.h (see pcs.h).  Reference: kzg/src/pcs.rs, commit/src/{pcs,domain}.rs.
#include "pcs.h"

#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <array>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <map>
#include <mutex>
#include <thread>

namespace eon_host {

void check(eon_ctx* ctx, int rc, const char* what) {
    if (rc == EON_OK) return;
    const char* msg = ctx ? eon_last_error(ctx) : nullptr;
    throw Error(rc, std::string(what) + ": " + (msg ? msg : "error"));
}

static void hip_check(hipError_t e, const char* what) {
    if (e != hipSuccess) throw Error(e == hipErrorOutOfMemory ? EON_E_OOM : EON_E_DEVICE,
                                     std::string(what) + ": " + hipGetErrorString(e));
}

// Freed buffers are kept (per device, exact size) for the next allocation of that size: a proof
// allocates the same matrices every time (the LDE alone is 11 GB at the headline size), and
// hipMalloc/hipFree of them per proof costs more than keeping them resident.  Capped at
// CACHE_CAP bytes; dropped wholesale when an allocation fails.
namespace {
constexpr uint64_t CACHE_CAP = 48ull << 30;
std::mutex cache_mu;
std::multimap<std::pair<int, uint64_t>, void*> cache;
uint64_t cached_bytes = 0;

void* cache_take(uint64_t bytes) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::lock_guard<std::mutex> lk(cache_mu);
    auto it = cache.find({dev, bytes});
    if (it == cache.end()) return nullptr;
    void* p = it->second;
    cache.erase(it);
    cached_bytes -= bytes;
    return p;
}

void cache_put(void* p, uint64_t bytes) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    {
        std::lock_guard<std::mutex> lk(cache_mu);
        if (cached_bytes + bytes <= CACHE_CAP) {
            cache.emplace(std::make_pair(dev, bytes), p);
            cached_bytes += bytes;
            return;
        }
    }
    (void)hipFree(p);
}

void cache_drop() {
    std::lock_guard<std::mutex> lk(cache_mu);
    for (auto& kv : cache) (void)hipFree(kv.second);
    cache.clear();
    cached_bytes = 0;
}
}  // namespace

DeviceBuffer::DeviceBuffer(uint64_t bytes) : bytes_(bytes) {
    if (!bytes) return;
    p_ = cache_take(bytes);
    if (p_) return;
    hipError_t e = hipMalloc(&p_, bytes);
    if (e == hipErrorOutOfMemory) {
        (void)hipGetLastError();
        cache_drop();
        e = hipMalloc(&p_, bytes);
    }
    hip_check(e, "hipMalloc");
}

DeviceBuffer::~DeviceBuffer() {
    if (p_) cache_put(p_, bytes_);
}

DeviceBuffer& DeviceBuffer::operator=(DeviceBuffer&& o) noexcept {
    if (this != &o) {
        if (p_) cache_put(p_, bytes_);
        p_ = o.p_;
        bytes_ = o.bytes_;
        o.p_ = nullptr;
        o.bytes_ = 0;
    }
    return *this;
}

DeviceMatrix DeviceMatrix::alloc(uint64_t height, uint32_t width) {
    DeviceMatrix m;
    m.owned = DeviceBuffer(std::max<uint64_t>(height * width, 1) * sizeof(eon_fr));
    m.height = height;
    m.width = width;
    return m;
}

DeviceMatrix DeviceMatrix::borrow(const eon_fr* p, uint64_t height, uint32_t width) {
    DeviceMatrix m;
    m.view = p;
    m.height = height;
    m.width = width;
    return m;
}

static uint32_t log2_ceil(uint64_t n) {
    uint32_t b = 0;
    while ((1ull << b) < n) b++;
    return b;
}

Domain Domain::create_disjoint_domain(uint64_t min_size) const {
    // shift * GENERATOR keeps the coset disjoint from the subgroup (domain.rs:155-168)
    return Domain{fr_mul(shift, fr_from_u64(5)), log2_ceil(min_size)};
}

std::vector<Domain> Domain::split_domains(uint32_t num_chunks) const {
    const uint32_t lc = log2_ceil(num_chunks);
    const Fr g = generator();
    std::vector<Domain> out;
    Fr s = shift;
    for (uint32_t i = 0; i < num_chunks; i++) {
        out.push_back(Domain{s, log_size - lc});
        s = fr_mul(s, g);
    }
    return out;
}

KzgPcs::KzgPcs(eon_ctx* ctx, uint64_t max_degree, const Fr& srs_alpha) : ctx_(ctx), max_degree_(max_degree) {
    // init_srs_unsafe (params.rs:123-139): g1_powers[i] = alpha^i * G for i <= max_degree, made on
    // device and turned into fixed-base MSM bases without a host round trip
    const uint64_t n = max_degree + 1;
    DeviceBuffer pts(n * sizeof(eon_g1_affine));
    const eon_fr a = srs_alpha.abi();
    check(ctx_, eon_g1_srs_powers_dev(ctx_, &a, n, pts.as<eon_g1_affine>()), "eon_g1_srs_powers_dev");
    check(ctx_, eon_msm_bases_create_dev(ctx_, pts.as<eon_g1_affine>(), n, EON_MSM_PRECOMPUTE, &bases_),
          "eon_msm_bases_create_dev");
    check(ctx_, eon_ctx_synchronize(ctx_), "eon_ctx_synchronize");
    // the auxiliary context: its own non-blocking stream, so that its work overlaps this
    // context's even when that one runs on the legacy null stream
    const int dev = eon_ctx_device(ctx_);
    hipStream_t s = nullptr;
    if (eon_ctx_create(dev, &aux_) == EON_OK) {
        if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) == hipSuccess &&
            eon_ctx_set_stream(aux_, s) == EON_OK) {
            aux_stream_ = s;
        } else {
            if (s) (void)hipStreamDestroy(s);
            eon_ctx_destroy(aux_);
            aux_ = nullptr;
        }
    }
}

KzgPcs::~KzgPcs() {
    if (bases_) eon_msm_bases_destroy(bases_);
    if (aux_) eon_ctx_destroy(aux_);
    if (aux_stream_) (void)hipStreamDestroy(static_cast<hipStream_t>(aux_stream_));
}

Domain KzgPcs::natural_domain_for_degree(uint64_t degree) const {
    return Domain{Fr::one(), degree > 1 ? log2_ceil(degree) : 0};
}

void KzgPcs::ensure_supported(uint64_t degree) const {
    if (degree > max_degree_)
        throw Error(EON_E_DEGREE_TOO_LARGE,
                    "degree " + std::to_string(degree) + " > max " + std::to_string(max_degree_));
}

void KzgPcs::commit_coeffs(std::vector<std::pair<Domain, DeviceMatrix>> evaluations,
                           std::vector<MatrixProverData>& data) {
    for (auto& [domain, evals] : evaluations) {
        const uint64_t h = evals.height;
        const uint32_t w = evals.width;
        if (h != domain.size()) throw Error(EON_E_SHAPE, "evaluation height must match domain size");
        ensure_supported(h > 0 ? h - 1 : 0);
        MatrixProverData d{domain, std::move(evals), DeviceMatrix::alloc(h, w), nullptr};
        const eon_fr s = domain.shift.abi();
        check(ctx_, eon_coset_idft_batch_dev(ctx_, d.evals.data(), d.coeffs.mutable_data(), h, w, &s),
              "coset_idft_batch");
        data.push_back(std::move(d));
    }
    check(ctx_, eon_ctx_synchronize(ctx_), "coset_idft_batch");
}

void KzgPcs::commit_columns(std::vector<MatrixProverData>& data, size_t first,
                            std::vector<std::vector<eon_g1_affine>>& commitments) {
    for (size_t k = first; k < data.size(); k++) {
        MatrixProverData& d = data[k];
        const uint64_t h = d.coeffs.height;
        const uint32_t w = d.coeffs.width;
        std::vector<eon_g1_affine> cm(w);
        // the column MSMs keep their sorted digits for the openings (KzgPcs::open)
        eon_msm_scalars* prep = nullptr;
        check(ctx_, eon_msm_g1_columns_prepare_dev(ctx_, bases_, d.coeffs.data(), h, w, cm.data(), &prep),
              "commit_column");
        d.prepared.reset(prep);
        commitments.push_back(std::move(cm));
    }
}

void KzgPcs::commit(std::vector<std::pair<Domain, DeviceMatrix>> evaluations,
                    std::vector<std::vector<eon_g1_affine>>& commitments, std::vector<MatrixProverData>& data) {
    const size_t first = data.size();
    commit_coeffs(std::move(evaluations), data);
    commit_columns(data, first, commitments);
}

DeviceMatrix KzgPcs::get_evaluations_on_domain(const std::vector<MatrixProverData>& data, size_t idx,
                                               const Domain& domain, bool aux) {
    eon_ctx* ctx = aux && aux_live() ? aux_ : ctx_;
    const MatrixProverData& m = data.at(idx);
    if (m.domain == domain) return DeviceMatrix::borrow(m.evals.data(), m.evals.height, m.evals.width);
    if (domain.log_size < m.domain.log_size)
        throw Error(EON_E_SHAPE, "evaluation domain smaller than the committed domain");
    const uint32_t added = domain.log_size - m.domain.log_size;
    DeviceMatrix out = DeviceMatrix::alloc(m.coeffs.height << added, m.coeffs.width);
    const eon_fr s = domain.shift.abi();
    check(ctx,
          eon_coset_dft_padded_batch_dev(ctx, m.coeffs.data(), out.mutable_data(), m.coeffs.height, m.coeffs.width,
                                         added, &s, EON_ORDER_NATURAL),
          "get_evaluations_on_domain");
    if (ctx != ctx_) check(ctx, eon_ctx_synchronize(ctx), "get_evaluations_on_domain");
    return out;
}

void KzgPcs::commit_quotient(const Domain& quotient_domain, const DeviceMatrix& quotient_evals, uint32_t num_chunks,
                             std::vector<std::vector<eon_g1_affine>>& commitments,
                             std::vector<MatrixProverData>& data, const std::vector<uint32_t>* only) {
    // split_evals: chunk c holds rows {i * num_chunks + c} (a strided column gather on device)
    if (quotient_evals.width != 1 || quotient_evals.height != quotient_domain.size() || num_chunks == 0 ||
        quotient_evals.height % num_chunks)
        throw Error(EON_E_SHAPE, "quotient evaluations must be one column over the quotient domain");
    const uint64_t rows = quotient_evals.height / num_chunks;
    hipStream_t st = static_cast<hipStream_t>(eon_ctx_stream(ctx_));
    std::vector<std::pair<Domain, DeviceMatrix>> chunks;
    const std::vector<Domain> doms = quotient_domain.split_domains(num_chunks);
    std::vector<uint32_t> all(num_chunks);
    for (uint32_t c = 0; c < num_chunks; c++) all[c] = c;
    for (const uint32_t c : only ? *only : all) {
        if (c >= num_chunks) throw Error(EON_E_ARG, "quotient chunk index out of range");
        DeviceMatrix m = DeviceMatrix::alloc(rows, 1);
        hip_check(hipMemcpy2DAsync(m.mutable_data(), sizeof(eon_fr), quotient_evals.data() + c,
                                   sizeof(eon_fr) * num_chunks, sizeof(eon_fr), rows, hipMemcpyDeviceToDevice, st),
                  "split_evals");
        chunks.emplace_back(doms[c], std::move(m));
    }
    commit(std::move(chunks), commitments, data);
}

std::vector<Opened> KzgPcs::open(const std::vector<OpenRound>& rounds) {
    for (const OpenRound& r : rounds) {
        if (r.data->size() != r.points.size()) throw Error(EON_E_SHAPE, "one point list per matrix");
        for (const MatrixProverData& m : *r.data)
            if (!m.prepared) throw Error(EON_E_ARG, "open: matrix committed without its prepared digits");
    }
    using Key = std::pair<uint64_t, std::array<uint64_t, 4>>;
    auto key_of = [](uint64_t n, const Fr& z) {
        const eon_fr za = z.abi();
        return Key(n, std::array<uint64_t, 4>{za.l[0], za.l[1], za.l[2], za.l[3]});
    };
    // opening bases per distinct (height, point), in order of first use; shared by every matrix
    // opened there (the trace and the quotient chunks at zeta)
    std::vector<Key> keys;
    std::map<Key, eon_msm_bases*> bases_at;
    struct BasesGuard {
        std::map<Key, eon_msm_bases*>& m;
        ~BasesGuard() {
            for (auto& kv : m)
                if (kv.second) eon_msm_bases_destroy(kv.second);
        }
    } guard{bases_at};
    for (const OpenRound& r : rounds)
        for (size_t m = 0; m < r.data->size(); m++)
            for (const Fr& z : r.points[m]) {
                const Key k = key_of((*r.data)[m].coeffs.height, z);
                if (bases_at.emplace(k, nullptr).second) keys.push_back(k);
            }
    auto build = [&](eon_ctx* c, const std::vector<Key>& ks) {
        std::map<uint64_t, std::vector<eon_fr>> by_height;
        for (const Key& k : ks) by_height[k.first].push_back(eon_fr{{k.second[0], k.second[1], k.second[2], k.second[3]}});
        for (auto& [n, zs] : by_height) {
            std::vector<eon_msm_bases*> made(zs.size(), nullptr);
            check(c, eon_kzg_opening_bases_create_many(c, bases_, n, zs.data(), (uint32_t)zs.size(), made.data()),
                  "opening bases");
            for (size_t t = 0; t < zs.size(); t++)
                bases_at[Key(n, std::array<uint64_t, 4>{zs[t].l[0], zs[t].l[1], zs[t].l[2], zs[t].l[3]})] = made[t];
        }
    };
    hipStream_t st = static_cast<hipStream_t>(eon_ctx_stream(ctx_));
    std::vector<Opened> out(rounds.size());
    // f(z) of every column at every point (the remainder of quotient_and_eval, util.rs:100-111):
    // enqueued on the auxiliary context, whose HBM-bound passes over the coefficients run beside
    // the VALU-bound opening-bases construction; read back after the witnesses
    eon_ctx* vctx = aux_live() ? aux_ : ctx_;
    hipStream_t vst = static_cast<hipStream_t>(eon_ctx_stream(vctx));
    std::vector<std::vector<DeviceBuffer>> vals(rounds.size());
    struct DrainOnExit {  // an error path must not free `vals` under the kernels writing them
        hipStream_t s;
        ~DrainOnExit() { (void)hipStreamSynchronize(s); }
    } drain{vst};
    for (size_t r = 0; r < rounds.size(); r++) {
        const auto& data = *rounds[r].data;
        out[r].values.resize(data.size());
        out[r].witnesses.resize(data.size());
        for (size_t m = 0; m < data.size(); m++) {
            const MatrixProverData& md = data[m];
            const std::vector<Fr>& pts = rounds[r].points[m];
            const uint32_t w = md.coeffs.width;
            out[r].values[m].resize(pts.size());
            out[r].witnesses[m].resize(pts.size());
            vals[r].emplace_back(std::max<uint64_t>(pts.size() * w, 1) * sizeof(eon_fr));
            std::vector<eon_fr> zs(pts.size());
            for (size_t p = 0; p < pts.size(); p++) zs[p] = pts[p].abi();
            check(vctx,
                  eon_eval_columns_dev(vctx, md.coeffs.data(), md.coeffs.height, w, zs.data(), (uint32_t)zs.size(),
                                       vals[r].back().as<eon_fr>()),
                  "opened values");
        }
    }
    auto collect_values = [&] {
        for (size_t r = 0; r < rounds.size(); r++)
            for (size_t m = 0; m < rounds[r].data->size(); m++) {
                const size_t np = rounds[r].points[m].size();
                const uint32_t w = (*rounds[r].data)[m].coeffs.width;
                std::vector<eon_fr> hv(np * w);
                hip_check(hipMemcpyAsync(hv.data(), vals[r][m].get(), hv.size() * sizeof(eon_fr),
                                         hipMemcpyDeviceToHost, vst),
                          "opened values");
                hip_check(hipStreamSynchronize(vst), "opened values");
                for (size_t p = 0; p < np; p++)
                    out[r].values[m][p].assign(hv.begin() + p * w, hv.begin() + (p + 1) * w);
            }
    };
    // witnesses of the (matrix, point) pairs whose bases are ready, every point of a matrix in
    // one run over its prepared digits
    std::vector<std::vector<std::vector<bool>>> done(rounds.size());
    for (size_t r = 0; r < rounds.size(); r++)
        for (size_t m = 0; m < rounds[r].points.size(); m++) done[r].emplace_back(rounds[r].points[m].size(), false);
    auto run_ready = [&] {
        for (size_t r = 0; r < rounds.size(); r++)
            for (size_t m = 0; m < rounds[r].data->size(); m++) {
                const MatrixProverData& md = (*rounds[r].data)[m];
                const uint32_t w = md.coeffs.width;
                std::vector<size_t> ps;
                std::vector<const eon_msm_bases*> hb;
                for (size_t p = 0; p < rounds[r].points[m].size(); p++) {
                    eon_msm_bases* b = bases_at.at(key_of(md.coeffs.height, rounds[r].points[m][p]));
                    if (done[r][m][p] || !b) continue;
                    ps.push_back(p);
                    hb.push_back(b);
                }
                if (ps.empty()) continue;
                std::vector<eon_g1_affine> wits(ps.size() * w);
                check(ctx_,
                      eon_msm_g1_columns_prepared(ctx_, hb.data(), (uint32_t)hb.size(), md.prepared.get(), wits.data()),
                      "witnesses");
                for (size_t q = 0; q < ps.size(); q++) {
                    out[r].witnesses[m][ps[q]].assign(wits.begin() + q * w, wits.begin() + (q + 1) * w);
                    done[r][m][ps[q]] = true;
                }
            }
    };
    build(ctx_, keys);
    run_ready();
    collect_values();
    return out;
}

}  // namespace eon_host
