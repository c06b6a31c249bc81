// Generic AIR quotient: quotient_values (eon-uni-stark/src/prover.rs:539-709) for ANY AIR whose
// constraints arrive as the symbolic DAG get_symbolic_constraints returns
// (eon-uni-stark/src/symbolic_builder.rs:72-126; SymbolicExpression, symbolic_expression.rs:78-145).
//
// Host side (eon_air_program_create): the DAG is value-numbered (hash-consing: identical leaves,
// constants by value, commutative + and * with sorted operands), scheduled constraint by
// constraint in the folder's order (each constraint's not-yet-computed sub-DAG in post-order, then
// its ASSERT), and register-allocated by liveness (a register is reused right after its last read).
// Leaves are operand modes, not instructions: trace column of the local / next row, a constant
// (program constants, then the public values), a selector.  degree_multiple follows
// symbolic_expression.rs:171-190, get_log_quotient_degree symbolic_builder.rs:15-43.
//
// Device side (k_air_quotient): one thread per quotient-domain row i runs the program with its
// row window (local = row i, next = row (i + 2^qd) mod Q, vertically_packed_row_pair,
// matrix/src/lib.rs:392-411), the selectors of selectors_on_coset at i, and the folder's
// accumulator as a Horner chain acc = acc * alpha + C_k (folder.rs:81-85 with the reversed alpha
// powers of prover.rs:578-579), stepped two constraints at a time (acc alpha^2 + C_k alpha +
// C_k+1: two limb products, one Montgomery reduction).  out[i] = acc * inv_vanishing[i] (prover.rs:699).  Every lane of
// a wave executes the same instruction (uniform program counter: scalar instruction fetch, the next
// instruction's fetch issued before the current one executes, no divergence).  A value read only
// by the next instruction is forwarded in registers (operand mode M_PREV, no register-file round
// trip).  Arithmetic is radix 2^29 with compiler-tracked value bounds (below).  Registers 0 and 1
// live in VGPRs, the rest in LDS (three planes: two 16-byte, one 4-byte; conflict-free accesses)
// sized by the program's register count, or in a global buffer for very large programs.
#include <algorithm>
#include <cstdlib>
#include <map>
#include <tuple>
#include <vector>

#include "field29.h"
#include "quotient.h"

using namespace eon;

namespace {

enum : uint32_t { OP_ADD = 0, OP_SUB = 1, OP_MUL = 2, OP_NEG = 3, OP_ASSERT = 4, OP_NOP = 5, OP_SQR = 6 };
// OP_SQR: a product of a value by itself (x * x after hash-consing), sqr29's 45 limb products
// instead of 81
// op word: opcode (bits 0-3) | OP_RED (the result is brought below 2p by reduce_top29) | K << K_SHIFT
// (OP_SUB / OP_NEG: the multiple of p added, at least the subtrahend's bound)
constexpr uint32_t OP_MASK = 0xf, OP_RED = 0x10, K_SHIFT = 8;
// OP_ASSERT's kind (in the K field): the constraints are folded in pairs, acc alpha^2 + C_k alpha +
// C_k+1 with one reduction (mul29_sum2): the first of a pair is held (AS_PEND), the second folds
// both (AS_PAIR).  With an odd count the first constraint opens the chain alone (AS_INIT: acc = C,
// acc alpha + C from acc = 0).
enum : uint32_t { AS_INIT = 0, AS_PEND = 1, AS_PAIR = 2 };
// Value bounds.  Every value is held in radix 2^29 as x 2^261 ("29-Montgomery", field29.h) with
// normalised limbs and a value below B p, B tracked per value by the compiler: products B = 2, a
// sum B_a + B_b, a difference B_a + K.  A result whose bound would exceed B_MAX is reduced in the
// same instruction (OP_RED: reduce_top29, B = 2), so every computed operand is below B_MAX p; with
// the raw leaves below (OPND_RAW) every product stays below 160 p^2, inside mul29's 167 p^2, and a
// reduced input below 64 p < 2^261.  The folder's accumulator stays below (2 + B_RAW) p.
constexpr uint32_t B_MAX = 12;
// A leaf (trace cell, constant, selector) is loaded either reduced (shl5_to261, B = 2) or raw
// (shl5_raw, B = 32: the reduction skipped) -- chosen per use by the compiler (OPND_RAW): raw
// wherever the reader allows it (a sum or difference, whose result is reduced anyway when it
// exceeds B_MAX, a constraint value, one side of a product whose other side is < 5p), so a
// two-leaf sum costs one reduction instead of two.  The subtrahend multiple K then reaches 32.
constexpr uint32_t B_RAW = 32, K_MAX = 32;
// Registers 0 and 1 -- the busiest: the allocator hands out the lowest free register -- are held in
// VGPRs, the others in LDS (36 bytes each, MemRegs).  At the Poseidon2-AIR's 5 registers and 256
// threads per block that is 27 KB of LDS per block instead of 45, so occupancy is set by the VGPRs
// (4 waves per SIMD) instead of the LDS (3).  Measured (round 4, profiles/r04/s13): all registers
// in LDS 15.6 ms, one in VGPRs 13.6, two 12.9; three spill; 64- or 128-thread blocks and a
// 5-wave launch bound (spills) are slower or equal.
constexpr uint32_t AIR_VREGS = 2, AIR_BLOCK = 256;
// operand = mode << 29 | index
enum : uint32_t { M_REG = 0, M_LOCAL = 1, M_NEXT = 2, M_CONST = 3, M_FIRST = 4, M_LAST = 5, M_TRANS = 6, M_PREV = 7 };
constexpr uint32_t OPND_RAW = 1u << 28, IDX_MASK = (1u << 28) - 1;
constexpr uint32_t NO_DST = ~0u;  // result only forwarded to the next instruction (M_PREV)

struct Instr {
    uint32_t op, dst, a, b;
};

// K p in normalised 29-bit limbs for K <= K_MAX (OP_SUB / OP_NEG); K is uniform, so its row is
// read with scalar loads
struct KpTable {
    uint32_t l[K_MAX + 1][9];
    constexpr KpTable() : l{} {
        for (uint32_t k = 0; k <= K_MAX; k++) {
            uint64_t c = 0;
            for (int i = 0; i < 9; i++) {
                c += (uint64_t)R29<FrP>::P[i] * k;
                l[k][i] = (uint32_t)(c & M29);
                c >>= 29;
            }
        }
    }
};
__device__ constexpr KpTable KP_TABLE{};

// a - b + K p, normalised (b < K p; a, b normalised: the signed column sums stay inside int32)
__device__ __forceinline__ F29 sub29_k(const F29& a, const F29& b, uint32_t k) {
    const uint32_t* kp = KP_TABLE.l[k];
    F29 r;
    int32_t c = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) {
        const int32_t t = (int32_t)(a.l[i] + kp[i]) - (int32_t)b.l[i] + c;
        r.l[i] = (uint32_t)t & M29;
        c = t >> 29;  // arithmetic: -1, 0 or 1
    }
    return r;
}

// a trace cell, constant or selector (canonical, x 2^256) as x 2^261: below 2p, or below 32p
// unreduced when the operand is marked raw (the flag is uniform: a scalar branch)
__device__ __forceinline__ F29 ld29(const Fr* p, bool raw) {
    const F29 x = shl5_raw<FrP>(ld_pinned(p));
    return raw ? x : reduce_top29<FrP>(x);
}

// register file in LDS or in a global buffer: 36 bytes per register in three planes (limbs 0-3
// and 4-7 as 16-byte planes, limb 8 as a 4-byte one), conflict-free b128 / b32 accesses
struct MemRegs {
    uint4* base;     // plane j of register r at (2 r + j) stride
    uint32_t* top;   // limb 8 of register r at r stride
    uint64_t stride;
    __device__ __forceinline__ F29 get(uint32_t r) const {
        const uint4 a = base[(uint64_t)(2 * r) * stride], b = base[(uint64_t)(2 * r + 1) * stride];
        F29 x;
        x.l[0] = a.x; x.l[1] = a.y; x.l[2] = a.z; x.l[3] = a.w;
        x.l[4] = b.x; x.l[5] = b.y; x.l[6] = b.z; x.l[7] = b.w;
        x.l[8] = top[(uint64_t)r * stride];
        return x;
    }
    __device__ __forceinline__ void set(uint32_t r, const F29& x) {
        base[(uint64_t)(2 * r) * stride] = make_uint4(x.l[0], x.l[1], x.l[2], x.l[3]);
        base[(uint64_t)(2 * r + 1) * stride] = make_uint4(x.l[4], x.l[5], x.l[6], x.l[7]);
        top[(uint64_t)r * stride] = x.l[8];
    }
};

struct Window {
    const Fr* local;
    const Fr* next;
    const F29* table;  // program constants, then public values: x 2^261 (< 2p), converted on the host
    const Fr* sels;   // is_first_row | is_last_row | is_transition, q each (null if unused)
    uint64_t row, q;
};

// the registers held in VGPRs: register j < AIR_VREGS is hj (named values, not an array: an array
// indexed by the register number went to scratch); the register number is uniform, so the choice
// is a scalar branch
static_assert(AIR_VREGS <= 4, "at most four registers in VGPRs");
struct Hot {
    F29 h0, h1, h2, h3;
};
__device__ __forceinline__ bool hot_get(const Hot& h, uint32_t i, F29& x) {
    if (i >= AIR_VREGS) return false;
    // limb-wise value selects (a branch per register was merged into a load through a selected
    // pointer, which put the registers in scratch)
#pragma unroll
    for (int k = 0; k < 9; k++) {
        uint32_t v = h.h0.l[k];
        if (AIR_VREGS > 1) v = i == 1 ? h.h1.l[k] : v;
        if (AIR_VREGS > 2) v = i == 2 ? h.h2.l[k] : v;
        if (AIR_VREGS > 3) v = i == 3 ? h.h3.l[k] : v;
        x.l[k] = v;
    }
    return true;
}
__device__ __forceinline__ bool hot_set(Hot& h, uint32_t i, const F29& x) {
    if (i >= AIR_VREGS) return false;
#pragma unroll
    for (int k = 0; k < 9; k++) {
        h.h0.l[k] = i == 0 ? x.l[k] : h.h0.l[k];
        if (AIR_VREGS > 1) h.h1.l[k] = i == 1 ? x.l[k] : h.h1.l[k];
        if (AIR_VREGS > 2) h.h2.l[k] = i == 2 ? x.l[k] : h.h2.l[k];
        if (AIR_VREGS > 3) h.h3.l[k] = i == 3 ? x.l[k] : h.h3.l[k];
    }
    return true;
}

// One load site for every trace-cell / selector mode and one second-operand fetch per slot: the
// kernel body (four slots written out) is 61 KB instead of 103 (round 6; the instruction cache hit
// 99.7 % before, and the time did not change: 11.69 vs 11.64 ms, profiles/r06/s7)

template <class RF>
__device__ __forceinline__ F29 fetch(uint32_t opnd, const RF& rf, const F29& prev, const Hot& hot, const Window& w) {
    const uint32_t i = opnd & IDX_MASK;
    const bool raw = (opnd & OPND_RAW) != 0;
    const uint32_t m = opnd >> 29;
    if (m == M_PREV) return prev;
    if (m == M_CONST) return w.table[i];  // uniform index: scalar loads, no conversion
    if (m == M_REG) {
        F29 x;
        if (hot_get(hot, i, x)) return x;
        return rf.get(i - AIR_VREGS);
    }
    // local / next row cell or a selector: the address picked by the (uniform) mode, one load
    const Fr* p = m == M_LOCAL ? w.local + i
                  : m == M_NEXT ? w.next + i
                                : w.sels + (uint64_t)(m - M_FIRST) * w.q + w.row;
    return ld29(p, raw);
}

// The program is fetched in blocks of CODE_BLOCK instructions (one 64-byte scalar load each; the
// device copy is padded with OP_NOP to a whole block), the next block's load issued before the
// current block runs: the program (~130 KB for the Poseidon2-AIR) does not fit the scalar cache, so
// every fetch is an L2 round trip that an instruction-at-a-time loop waits on.
constexpr uint32_t CODE_BLOCK = 4;
struct CodeBlock {
    Instr i[CODE_BLOCK];
};

// The four slots of a block are unrolled, each with its own product per op kind.  One shared body
// (the slot's words picked by scalar selects, one product for MUL and ASSERT) measured slower,
// 15.8 vs 14.8 ms for the Poseidon2-AIR at 2^18 rows (round 4, profiles/r04/s7): not kept.
template <class RF>
__device__ __forceinline__ void exec1(const Instr& in, RF& rf, const Window& w, const F29& alpha,
                                      const F29& alpha2, F29& acc, F29& pend, F29& prev, Hot& hot) {
    const uint32_t opc = in.op & OP_MASK;
    if (opc == OP_NOP) return;
    const F29 x = fetch(in.a, rf, prev, hot, w);
    if (opc == OP_ASSERT) {  // folder.rs:81-85, alpha powers reversed
        const uint32_t kind = in.op >> K_SHIFT;
        if (kind == AS_PAIR)  // acc < 34p, pend < 32p: acc alpha^2 + pend alpha < 132 p^2
            acc = add29_lazy(mul29_sum2_u<FrP>(alpha2, acc, alpha, pend), x);
        else if (kind == AS_PEND)
            pend = x;
        else
            acc = x;
        return;
    }
    F29 r;
    if (opc == OP_SQR) {
        r = sqr29<FrP>(x);
    } else {
        F29 a = x, b;
        if (opc == OP_NEG) {  // 0 - x + K p
            b = x;
#pragma unroll
            for (int i = 0; i < 9; i++) a.l[i] = 0;
        } else {
            b = fetch(in.b, rf, prev, hot, w);
        }
        if (opc == OP_MUL) {
            r = mul29<FrP>(a, b);
        } else {
            r = opc == OP_ADD ? add29_norm(a, b) : sub29_k(a, b, in.op >> K_SHIFT);
            if (in.op & OP_RED) r = reduce_top29<FrP>(r);
        }
    }
    prev = r;
    if (in.dst == NO_DST || hot_set(hot, in.dst, r)) return;
    rf.set(in.dst - AIR_VREGS, r);
}

template <class RF>
__device__ __forceinline__ void run_program(const CodeBlock* __restrict__ code, uint32_t n_blocks, RF& rf,
                                            const Window& w, const F29& alpha, F29& acc) {
    if (n_blocks == 0) return;
    const F29 alpha2 = uniform29(sqr29<FrP>(alpha));
    F29 prev, pend;
    Hot hot;
#pragma unroll
    for (int i = 0; i < 9; i++) prev.l[i] = pend.l[i] = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) hot.h0.l[i] = hot.h1.l[i] = hot.h2.l[i] = hot.h3.l[i] = 0;
    CodeBlock nx = code[0];
    for (uint32_t bk = 0; bk < n_blocks; bk++) {
        const CodeBlock cur = nx;
        if (bk + 1 < n_blocks) nx = code[bk + 1];  // in flight while this block runs
        // the four slots written out: a loop over them is left rolled by the compiler at this body
        // size, and the block then goes through scratch to be indexed
        auto slot = [&](const Instr& raw) __attribute__((always_inline)) {
            const Instr in{(uint32_t)__builtin_amdgcn_readfirstlane(raw.op),
                           (uint32_t)__builtin_amdgcn_readfirstlane(raw.dst),
                           (uint32_t)__builtin_amdgcn_readfirstlane(raw.a),
                           (uint32_t)__builtin_amdgcn_readfirstlane(raw.b)};
            exec1(in, rf, w, alpha, alpha2, acc, pend, prev, hot);
        };
        static_assert(CODE_BLOCK == 4, "four slots below");
        slot(cur.i[0]);
        slot(cur.i[1]);
        slot(cur.i[2]);
        slot(cur.i[3]);
    }
}

// MODE 0: registers in LDS; 1: in the global buffer `gregs` (n_regs 36-byte registers per row)
template <int MODE>
__global__ void __launch_bounds__(AIR_BLOCK) k_air_quotient(const CodeBlock* __restrict__ code, uint32_t n_blocks,
                                                      uint32_t n_regs, const Fr* __restrict__ lde, uint32_t width,
                                                      uint64_t q, uint64_t next_step, const F29* __restrict__ table,
                                                      const Fr* __restrict__ sels, const Fr* __restrict__ inv_van,
                                                      uint32_t nr_mask, Fr alpha, Fr* __restrict__ out,
                                                      uint4* __restrict__ gregs) {
    extern __shared__ uint4 lds_regs[];
    const uint64_t row = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (row >= q) return;
    Window w{lde + row * width, lde + ((row + next_step) & (q - 1)) * width, table, sels, row, q};
    F29 acc;
#pragma unroll
    for (int i = 0; i < 9; i++) acc.l[i] = 0;
    const uint32_t n_mem = n_regs > AIR_VREGS ? n_regs - AIR_VREGS : 0;  // registers in memory
    MemRegs rf;
    if (MODE == 0) {
        rf.base = lds_regs + threadIdx.x;
        rf.top = reinterpret_cast<uint32_t*>(lds_regs + 2ull * n_mem * blockDim.x) + threadIdx.x;
        rf.stride = blockDim.x;
    } else {
        rf.base = gregs + row;
        rf.top = reinterpret_cast<uint32_t*>(gregs + 2ull * n_mem * q) + row;
        rf.stride = q;
    }
    run_program(code, n_blocks, rf, w, uniform29(shl5_to261<FrP>(alpha)), acc);
    // acc (x 2^261, < (2 + B_RAW) p, limbs < 2^30) times inv_vanishing in the ABI form: x 2^261 y 2^256 2^-261
    // = x y 2^256 (prover.rs:699)
    const F29 r = mul29<FrP>(acc, unpack29(ld_pinned(inv_van + (row & nr_mask))));
    st_vec(out + row, pack29<FrP>(canon29<FrP>(r)));
}

}  // namespace

struct eon_air_program {
    eon_ctx* ctx = nullptr;
    uint32_t width = 0, n_public = 0, n_constraints = 0, max_degree = 0, n_regs = 0, n_consts = 0;
    bool uses_sels = false;
    std::vector<Instr> code;
    std::vector<Fr> consts;
    DevBuf d_code, d_table, d_sels, d_regs;
    std::vector<Fr> staged;  // host copy of the table for the current launch
    std::vector<F29> staged29;  // the same in the device's form (x 2^261, < 2p)
};

namespace {

int finish(eon_ctx* ctx, const Status& s) {
    if (s.bad()) ctx->last_error = s.msg;
    return s.code;
}

struct Leaf {
    uint32_t kind, a, b;
};

// compile nodes -> program; see the file comment
Status compile(eon_air_program* p, const eon_sym_node* nodes, uint32_t n_nodes, const eon_fr* consts,
               uint32_t n_consts, const uint32_t* roots, uint32_t n_roots) {
    // operand indices are 28 bits (bit 28 is OPND_RAW): a wider main-column index, constant slot
    // or public slot would set the raw flag and read the wrong leaf
    if (p->width > IDX_MASK || (uint64_t)n_consts + p->n_public > IDX_MASK)
        return Status::err(EON_E_SHAPE, "trace width and constant + public slots must each be < 2^28");
    // value numbering
    std::vector<uint32_t> vn(n_nodes);
    std::vector<uint32_t> degree(n_nodes);
    struct Val {
        uint32_t op;            // OP_* for computed values, ~0u for leaves
        uint32_t a, b;          // operand value numbers (computed) / operand code (leaf)
    };
    std::vector<Val> vals;
    std::map<std::tuple<uint32_t, uint32_t, uint32_t>, uint32_t> memo;
    std::map<std::vector<uint32_t>, uint32_t> const_slot;  // canonical limbs -> table index
    auto intern = [&](uint32_t op, uint32_t a, uint32_t b) -> uint32_t {
        auto key = std::make_tuple(op, a, b);
        auto it = memo.find(key);
        if (it != memo.end()) return it->second;
        const uint32_t id = (uint32_t)vals.size();
        vals.push_back({op, a, b});
        memo.emplace(key, id);
        return id;
    };
    constexpr uint32_t LEAF = ~0u;
    for (uint32_t i = 0; i < n_nodes; i++) {
        const eon_sym_node& nd = nodes[i];
        auto operand = [&](uint32_t j) -> Status {
            if (j >= i) return Status::err(EON_E_ARG, "node " + std::to_string(i) + ": operand must precede it");
            return Status::ok();
        };
        switch (nd.kind) {
            case EON_SYM_CONSTANT: {
                if (nd.a >= n_consts) return Status::err(EON_E_ARG, "constant index out of range");
                const Fr c = fr_from_abi(&consts[nd.a]);
                if (!fr_is_canonical(c)) return Status::err(EON_E_ARG, "constant is not a canonical Fr");
                std::vector<uint32_t> key(c.v, c.v + 8);
                auto it = const_slot.find(key);
                uint32_t slot;
                if (it == const_slot.end()) {
                    slot = (uint32_t)p->consts.size();
                    p->consts.push_back(c);
                    const_slot.emplace(key, slot);
                } else {
                    slot = it->second;
                }
                vn[i] = intern(LEAF, M_CONST << 29 | slot, 0);
                degree[i] = 0;
                break;
            }
            case EON_SYM_MAIN:
                if (nd.a >= p->width || nd.b > 1) return Status::err(EON_E_ARG, "main variable out of range");
                vn[i] = intern(LEAF, (nd.b ? M_NEXT : M_LOCAL) << 29 | nd.a, 0);
                degree[i] = 1;
                break;
            case EON_SYM_PUBLIC:
                if (nd.a >= p->n_public) return Status::err(EON_E_ARG, "public value index out of range");
                vn[i] = intern(LEAF, 0xffffffffu, nd.a);  // resolved to a table slot below
                degree[i] = 0;
                break;
            case EON_SYM_IS_FIRST_ROW:
            case EON_SYM_IS_LAST_ROW:
            case EON_SYM_IS_TRANSITION: {
                const uint32_t m = nd.kind == EON_SYM_IS_FIRST_ROW ? M_FIRST
                                   : nd.kind == EON_SYM_IS_LAST_ROW ? M_LAST : M_TRANS;
                vn[i] = intern(LEAF, m << 29, 0);
                degree[i] = nd.kind == EON_SYM_IS_TRANSITION ? 0 : 1;
                break;
            }
            case EON_SYM_ADD:
            case EON_SYM_MUL: {
                EON_TRY(operand(nd.a));
                EON_TRY(operand(nd.b));
                uint32_t x = vn[nd.a], y = vn[nd.b];
                if (x > y) std::swap(x, y);  // commutative
                vn[i] = intern(nd.kind == EON_SYM_ADD ? OP_ADD : OP_MUL, x, y);
                degree[i] = nd.kind == EON_SYM_ADD ? std::max(degree[nd.a], degree[nd.b])
                                                   : degree[nd.a] + degree[nd.b];
                break;
            }
            case EON_SYM_SUB:
                EON_TRY(operand(nd.a));
                EON_TRY(operand(nd.b));
                vn[i] = intern(OP_SUB, vn[nd.a], vn[nd.b]);
                degree[i] = std::max(degree[nd.a], degree[nd.b]);
                break;
            case EON_SYM_NEG:
                EON_TRY(operand(nd.a));
                vn[i] = intern(OP_NEG, vn[nd.a], 0);
                degree[i] = degree[nd.a];
                break;
            case EON_SYM_PREPROCESSED:
            case EON_SYM_PERMUTATION:
            case EON_SYM_CHALLENGE:
                return Status::err(EON_E_ARG, "preprocessed / permutation (LogUp) / challenge variables are not "
                                              "supported by the generic quotient program");
            default:
                return Status::err(EON_E_ARG, "unknown node kind " + std::to_string(nd.kind));
        }
    }
    p->n_consts = (uint32_t)p->consts.size();
    // public values occupy the table slots after the constants
    for (auto& v : vals)
        if (v.op == LEAF && v.a == 0xffffffffu) v.a = M_CONST << 29 | (p->n_consts + v.b);
    for (auto& v : vals)
        if (v.op == LEAF) {
            const uint32_t m = v.a >> 29;
            if (m == M_FIRST || m == M_LAST || m == M_TRANS) p->uses_sels = true;
        }
    p->max_degree = 0;
    for (uint32_t k = 0; k < n_roots; k++) {
        if (roots[k] >= n_nodes) return Status::err(EON_E_ARG, "constraint index out of range");
        p->max_degree = std::max(p->max_degree, degree[roots[k]]);
    }
    // schedule: per constraint, post-order of its not-yet-emitted values, then ASSERT
    const uint32_t nv = (uint32_t)vals.size();
    std::vector<uint32_t> order;  // emitted computed values
    std::vector<char> done(nv, 0);
    std::vector<std::pair<uint32_t, uint32_t>> asserts;  // (position in order, value)
    for (uint32_t k = 0; k < n_roots; k++) {
        std::vector<std::pair<uint32_t, bool>> st{{vn[roots[k]], false}};
        while (!st.empty()) {
            auto [v, ready] = st.back();
            st.pop_back();
            if (done[v] || vals[v].op == LEAF) continue;
            if (!ready) {
                st.push_back({v, true});
                const uint32_t kids[2] = {vals[v].a, vals[v].op == OP_NEG ? LEAF : vals[v].b};
                for (int t = 1; t >= 0; t--)
                    if (kids[t] != LEAF && !done[kids[t]] && vals[kids[t]].op != LEAF) st.push_back({kids[t], false});
                continue;
            }
            done[v] = 1;
            order.push_back(v);
        }
        asserts.push_back({(uint32_t)order.size(), vn[roots[k]]});
    }
    // instruction stream: computed values interleaved with asserts
    struct Item {
        bool assert_;
        uint32_t v;
    };
    std::vector<Item> items;
    {
        size_t ai = 0;
        for (uint32_t pos = 0; pos <= order.size(); pos++) {
            while (ai < asserts.size() && asserts[ai].first == pos) items.push_back({true, asserts[ai++].second});
            if (pos < order.size()) items.push_back({false, order[pos]});
        }
    }
    // liveness: last read of each computed value
    std::vector<int64_t> last(nv, -1);
    for (size_t t = 0; t < items.size(); t++) {
        const Item& it = items[t];
        if (it.assert_) {
            last[it.v] = (int64_t)t;
        } else {
            const Val& x = vals[it.v];
            last[x.a] = (int64_t)t;
            if (x.op != OP_NEG) last[x.b] = (int64_t)t;
        }
    }
    // forwarding: a value whose only reader is the very next item never touches the register
    // file (the kernel keeps the previous result in registers, operand mode M_PREV)
    std::vector<int64_t> first_read(nv, -1);
    std::vector<uint32_t> n_readers(nv, 0);
    {
        std::vector<int64_t> last_reader(nv, -1);
        for (size_t t = 0; t < items.size(); t++) {
            const Item& it = items[t];
            uint32_t rd[2] = {it.v, LEAF};
            if (!it.assert_) {
                rd[0] = vals[it.v].a;
                rd[1] = vals[it.v].op == OP_NEG ? LEAF : vals[it.v].b;
            }
            for (uint32_t v : rd) {
                if (v == LEAF || vals[v].op == LEAF || last_reader[v] == (int64_t)t) continue;
                last_reader[v] = (int64_t)t;
                n_readers[v]++;
                if (first_read[v] < 0) first_read[v] = (int64_t)t;
            }
        }
    }
    std::vector<size_t> pos_of(nv, 0);
    for (size_t t = 0; t < items.size(); t++)
        if (!items[t].assert_) pos_of[items[t].v] = t;
    auto forwarded = [&](uint32_t v) {
        return vals[v].op != LEAF && n_readers[v] == 1 && first_read[v] == (int64_t)pos_of[v] + 1;
    };
    // register allocation (lowest free register; operands freed before the result is assigned)
    std::vector<uint32_t> reg(nv, ~0u);
    std::vector<uint32_t> free_regs;
    uint32_t n_regs = 0;
    auto opnd = [&](uint32_t v) {
        if (vals[v].op == LEAF) return vals[v].a;
        return forwarded(v) ? (M_PREV << 29) : (M_REG << 29 | reg[v]);
    };
    auto release = [&](uint32_t v, size_t t) {
        if (vals[v].op != LEAF && last[v] == (int64_t)t && reg[v] != ~0u) {
            free_regs.push_back(reg[v]);
            std::sort(free_regs.begin(), free_regs.end(), std::greater<uint32_t>());
        }
    };
    // value bounds in multiples of p (see B_MAX): products 2, leaves 2 or B_RAW as loaded, sums
    // and differences add up, a result above B_MAX is reduced by its own instruction
    std::vector<uint32_t> bound(nv, 2);
    auto is_leaf = [&](uint32_t v) { return vals[v].op == LEAF; };
    auto is_tleaf = [&](uint32_t v) { return is_leaf(v) && (vals[v].a >> 29) != M_CONST; };
    // assert kinds: pairs from the end of the chain, so an odd count leaves the first one alone
    uint32_t n_asserts = 0, seen = 0;
    for (const Item& it : items) n_asserts += it.assert_ ? 1 : 0;
    for (size_t t = 0; t < items.size(); t++) {
        const Item& it = items[t];
        if (it.assert_) {  // constraint values: < B_RAW p (raw leaf) or < B_MAX p
            const uint32_t odd = n_asserts & 1;
            const uint32_t kind = (odd && seen == 0) ? AS_INIT : ((seen - odd) % 2 == 0 ? AS_PEND : AS_PAIR);
            seen++;
            p->code.push_back({OP_ASSERT | kind << K_SHIFT, 0, opnd(it.v) | (is_tleaf(it.v) ? OPND_RAW : 0u), 0});
            release(it.v, t);
            continue;
        }
        const Val& x = vals[it.v];
        const bool unary = x.op == OP_NEG;
        // per use: the leaf operands raw unless a product's other side is too wide for it; constants
        // arrive reduced (the table is converted on the host), never raw
        bool raw_a = is_tleaf(x.a), raw_b = !unary && is_tleaf(x.b);
        const bool square = x.op == OP_MUL && x.a == x.b;  // sqr29: x < 12.9p, so never a raw leaf
        if (square) {
            raw_a = raw_b = false;
        } else if (x.op == OP_MUL) {
            if (raw_a && raw_b)
                raw_b = false;  // 32 x 2
            else if (raw_a && bound[x.b] * B_RAW > 160)
                raw_a = false;
            else if (raw_b && bound[x.a] * B_RAW > 160)
                raw_b = false;
        }
        const uint32_t ba = raw_a ? B_RAW : bound[x.a], bb = unary ? 0 : raw_b ? B_RAW : bound[x.b];
        uint32_t op = square ? OP_SQR : x.op, b = 2;
        if (x.op == OP_ADD) {
            b = ba + bb;
        } else if (x.op == OP_SUB) {
            op |= bb << K_SHIFT;  // + K p with K = the subtrahend's bound
            b = ba + bb;
        } else if (x.op == OP_NEG) {
            op |= ba << K_SHIFT;
            b = ba;
        }
        if (b > B_MAX) {
            op |= OP_RED;
            b = 2;
        }
        bound[it.v] = b;
        Instr in{op, 0, opnd(x.a) | (raw_a ? OPND_RAW : 0u),
                 (unary || square) ? 0u : opnd(x.b) | (raw_b ? OPND_RAW : 0u)};
        release(x.a, t);
        if (x.op != OP_NEG && x.b != x.a) release(x.b, t);
        if (last[it.v] < 0) continue;  // never read (cannot happen for reachable values)
        if (forwarded(it.v)) {
            in.dst = NO_DST;
            p->code.push_back(in);
            continue;
        }
        uint32_t r;
        if (!free_regs.empty()) {
            r = free_regs.back();
            free_regs.pop_back();
        } else {
            r = n_regs++;
        }
        reg[it.v] = r;
        in.dst = r;
        p->code.push_back(in);
    }
    p->n_regs = n_regs;
    if (n_regs > IDX_MASK) return Status::err(EON_E_SHAPE, "more than 2^28 - 1 registers");
    return Status::ok();
}

}  // namespace

extern "C" {

int eon_air_program_create(eon_ctx* ctx, const eon_sym_node* nodes, uint32_t n_nodes, const eon_fr* consts,
                           uint32_t n_consts, const uint32_t* constraints, uint32_t n_constraints, uint32_t width,
                           uint32_t n_public, eon_air_program** out) {
    if (!ctx) return EON_E_ARG;
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (hipSetDevice(ctx->device) != hipSuccess) return EON_E_DEVICE;
    Status s = [&]() -> Status {
        if (!out || (n_nodes && !nodes) || (n_consts && !consts) || (n_constraints && !constraints))
            return Status::err(EON_E_ARG, "null argument");
        auto* p = new eon_air_program();
        p->ctx = ctx;
        p->width = width;
        p->n_public = n_public;
        p->n_constraints = n_constraints;
        Status c = compile(p, nodes, n_nodes, consts, n_consts, constraints, n_constraints);
        if (c.bad()) {
            delete p;
            return c;
        }
        // device copy padded with OP_NOP to whole CODE_BLOCKs
        std::vector<Instr> padded(p->code);
        while (padded.size() % CODE_BLOCK) padded.push_back({OP_NOP, NO_DST, M_PREV << 29, 0});
        hipError_t e = p->d_code.ensure(std::max<size_t>(1, padded.size()) * sizeof(Instr));
        if (e == hipSuccess && !padded.empty())
            e = hipMemcpy(p->d_code.p, padded.data(), padded.size() * sizeof(Instr), hipMemcpyHostToDevice);
        if (e == hipSuccess) e = p->d_table.ensure(std::max<size_t>(1, p->n_consts + n_public) * sizeof(F29));
        if (e != hipSuccess) {
            p->d_code.release();
            p->d_table.release();
            delete p;
            EON_HIP(e);
        }
        *out = p;
        return Status::ok();
    }();
    return finish(ctx, s);
}

void eon_air_program_destroy(eon_air_program* p) {
    if (!p) return;
    std::lock_guard<std::mutex> lk(p->ctx->mu);
    (void)hipSetDevice(p->ctx->device);
    (void)hipStreamSynchronize(p->ctx->stream);
    for (DevBuf* b : {&p->d_code, &p->d_table, &p->d_sels, &p->d_regs}) b->release();
    delete p;
}

int eon_air_program_info(const eon_air_program* p, eon_air_program_stats* out) {
    if (!p || !out) return EON_E_ARG;
    out->width = p->width;
    out->num_public_values = p->n_public;
    out->num_constraints = p->n_constraints;
    out->max_constraint_degree = p->max_degree;
    out->num_instructions = (uint32_t)p->code.size();
    out->num_registers = p->n_regs;
    out->num_constants = p->n_consts;
    return EON_OK;
}

uint32_t eon_air_program_log_quotient_degree(const eon_air_program* p, uint32_t is_zk) {
    // symbolic_builder.rs:28-42: log2_ceil(max(max_degree + is_zk, 2) - 1)
    if (!p) return 0;
    const uint32_t d = std::max<uint32_t>(p->max_degree + (is_zk ? 1 : 0), 2) - 1;
    uint32_t b = 0;
    while ((1u << b) < d) b++;
    return b;
}

int eon_quotient_values_dev(eon_ctx* ctx, const eon_air_program* prog_c, const eon_fr* lde, uint32_t log_n,
                            uint32_t log_qd, const eon_fr* alpha, const eon_fr* publics, uint32_t n_public,
                            eon_fr* out) {
    if (!ctx || !prog_c) return EON_E_ARG;
    auto* prog = const_cast<eon_air_program*>(prog_c);  // device scratch only
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (hipSetDevice(ctx->device) != hipSuccess) return EON_E_DEVICE;
    Status s = [&]() -> Status {
        if (!lde || !alpha || !out || (n_public && !publics)) return Status::err(EON_E_ARG, "null argument");
        if (prog->ctx != ctx) return Status::err(EON_E_ARG, "program belongs to another context");
        if (n_public != prog->n_public)
            return Status::err(EON_E_SHAPE, "public value count differs from the program's");
        const uint32_t log_q = log_n + log_qd;
        EON_TRY(check_domains(log_n, log_q));
        const Fr al = fr_from_abi(alpha);
        if (!fr_is_canonical(al)) return Status::err(EON_E_ARG, "alpha is not a canonical Fr");
        const uint64_t q = 1ull << log_q;
        // constant table = program constants ++ public values
        prog->staged.assign(prog->consts.begin(), prog->consts.end());
        for (uint32_t i = 0; i < n_public; i++) {
            const Fr v = fr_from_abi(&publics[i]);
            if (!fr_is_canonical(v)) return Status::err(EON_E_ARG, "public value is not a canonical Fr");
            prog->staged.push_back(v);
        }
        if (!prog->staged.empty()) {
            prog->staged29.resize(prog->staged.size());
            for (size_t i = 0; i < prog->staged.size(); i++) prog->staged29[i] = shl5_to261<FrP>(prog->staged[i]);
            EON_HIP(hipMemcpyAsync(prog->d_table.p, prog->staged29.data(), prog->staged29.size() * sizeof(F29),
                                   hipMemcpyHostToDevice, ctx->stream));
            EON_HIP(hipStreamSynchronize(ctx->stream));  // `staged` is reused by the next launch
        }
        // quotient domain = trace domain (shift 1).create_disjoint_domain: shift GENERATOR
        // (commit/src/domain.rs:155-168); selectors_on_coset over it (prover.rs:563-564)
        const Fr g5 = from_u64<FrP>(5);
        const Fr* inv_van;
        if (prog->uses_sels) {
            EON_HIP(prog->d_sels.ensure(4 * q * sizeof(Fr)));
            EON_TRY(selectors_launch(ctx, log_n, log_q, g5, prog->d_sels.as<Fr>()));
            inv_van = prog->d_sels.as<Fr>() + 3 * q;
        } else {
            Fr *zh, *zh_inv;
            EON_TRY(vanishing_table(ctx, log_n, log_q, g5, &zh, &zh_inv));
            inv_van = zh_inv;
        }
        const uint32_t nr_mask = prog->uses_sels ? (uint32_t)(q - 1) : (1u << log_qd) - 1;
        // register file: LDS (block size shrinks with the register count), or global for very large
        // programs (EON_AIR_REGS=global forces it, for tests)
        static const bool force_global = [] {
            const char* e = getenv("EON_AIR_REGS");
            return e && std::string(e) == "global";
        }();
        // MemRegs: 36 bytes per register in memory
        const uint64_t per_thread = (uint64_t)(prog->n_regs > AIR_VREGS ? prog->n_regs - AIR_VREGS : 0) * 36;
        uint32_t block = AIR_BLOCK;
        while (block > 64 && block * per_thread > 64 * 1024) block /= 2;
        const int mode = !force_global && block * per_thread <= 160 * 1024 ? 0 : 1;
        if (mode != 0) block = AIR_BLOCK;
        if (mode == 1) EON_HIP(prog->d_regs.ensure(std::max<uint64_t>(1, q * per_thread)));
        const unsigned grid = (unsigned)((q + block - 1) / block);
        const size_t shmem = mode == 0 ? (size_t)block * per_thread : 0;
        // algorithmic 256-bit products per row: the program's multiplications, one acc * alpha per
        // constraint (ASSERT) and the final inv_vanishing product (additions, subtractions and
        // negations are not products)
        uint64_t products = 1;
        for (const Instr& in : prog->code) {
            const uint32_t opc = in.op & OP_MASK;
            products += (opc == OP_MUL || opc == OP_SQR || opc == OP_ASSERT) ? 1 : 0;
        }
        ctx->prof.begin("k_air_quotient", q * (uint64_t)prog->width * 32 + q * 32, ctx->stream, q * products);
        const CodeBlock* code = prog->d_code.as<CodeBlock>();
        const uint32_t n_blocks = (uint32_t)((prog->code.size() + CODE_BLOCK - 1) / CODE_BLOCK);
        const Fr* lde_f = reinterpret_cast<const Fr*>(lde);
        const Fr* sel = prog->uses_sels ? prog->d_sels.as<Fr>() : nullptr;
        Fr* out_f = reinterpret_cast<Fr*>(out);
        using KernelFn = void (*)(const CodeBlock*, uint32_t, uint32_t, const Fr*, uint32_t, uint64_t, uint64_t,
                                  const F29*, const Fr*, const Fr*, uint32_t, Fr, Fr*, uint4*);
        const KernelFn kern = mode == 0 ? k_air_quotient<0> : k_air_quotient<1>;
        if (mode == 0)  // per launch: the attribute is per device, and this context's device may
                        // differ from the one another context set it on
            EON_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        hipLaunchKernelGGL(kern, dim3(grid), dim3(block), shmem, ctx->stream, code, n_blocks, prog->n_regs, lde_f,
                           prog->width, q, 1ull << log_qd, prog->d_table.as<F29>(), sel, inv_van, nr_mask, al, out_f,
                           mode == 1 ? prog->d_regs.as<uint4>() : nullptr);
        ctx->prof.end(ctx->stream);
        EON_HIP(hipGetLastError());
        return Status::ok();
    }();
    return finish(ctx, s);
}

}  // extern "C"
