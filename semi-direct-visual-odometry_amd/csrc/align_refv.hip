// align_refv.hip — K2V: the reference's robust scale bit for bit with the residual vector resident in one CU's
// registers (median_mode SVO_MEDIAN_REFERENCE; three register layouts: LayA, vectors of <= 50 176 slots (the
// config-2 shape), LayB, <= 60 416 slots, LayC, <= 65 536; K2R in align_ref.hip takes larger ones).
//
// What it reproduces: Optimizer::tukeyWeighting (src/optimizer.cpp:485-514) takes sigma = 1.4826 * MAD with
// algorithm::computeMedian (src/algorithm.cpp:834-853) on the FULL residual vector (n_features * patch^2
// slots, feature-major, invisible slots = DBL_MAX): std::nth_element(vec, vec + n/2), then for an even total
// length (vec[n/2 - 1] + vec[n/2]) / 2 with vec[n/2 - 1] as libstdc++'s introselect left it; the MAD is the
// same call on |r_i - median| in the original order (:855-865).  The rounds are the parallel Hoare rounds of
// tests/cpp/introselect_model.cpp (checked there against the real std::nth_element):
//   median of three (first+1, first+S/2, last-1) moved to first, pivot p;
//   GE = positions in (first, last) with !(a < p), LE = positions in [first, last) with !(p < a);
//   the k-th GE from the left (L_k) and the k-th LE from the right (R_k) swap for k <= Ks,
//   Ks = max over split points t of min(#GE before t, #LE from t on); cut = min(L_{Ks+1}, R_{Ks}).
//
// Why registers.  A pair's vector is 50 000 doubles (400 KB) at config 2: more than the 160 KB of LDS, so
// K2R ran its large rounds through global scratch (three sweeps of the segment per round, ~6 MB of traffic
// per pair and level).  A CU's register file is 512 KB: one 512-thread workgroup (two waves per SIMD, 256
// VGPRs each) holds the whole vector, and every round works on registers.  Position q lives in lane q % 64 of
// wave (q / 64) % 8, row q / 512 ("step" q / 64 = 8 row + wave), so a segment [f, l) always spreads over all
// eight waves.  Per round (round 4's form):
//   1. classify: each wave walks its rows in quads with compile-time row numbers (refv_rows.h: the compares
//      name the data registers, no indexing mode), the GE / LE masks of row r go to lane r of four accumulators
//      (v_writelane), then four coalesced stores per 64 rows write the step records and the packed counts;  barrier
//   2. every wave reads the counts of all steps (lane r: the eight steps of row r), one DPP scan gives the row
//      prefixes; the crossing, Ks and the ranks L_{Ks+1}, R_{Ks}, L_{Ks} are ballots over the row lanes plus
//      a walk over one row's eight steps; the owners publish the pre-values the next round's pivot and
//      vec[nth - 1] need; the sources write the mailbox (LDS, slot k - 1), EXEC set to the row's side mask;  barrier
//   3. the kept side's targets take the mailbox values (EXEC-masked moves into the rows); all read the next
//      pivot's candidates.
// A mailbox larger than the layout's kMbCap swaps runs in chunks.  Segments of <= 1024 (LayC: 512) continue on wave 0 in
// its rows 0..15 (0..7) without barriers; the depth limit falls back to the restated heap select (adversarial inputs only).
// No global traffic but the two reads of K1's residuals per pair and level (one per pass).
#include "svo_internal.h"
#include "svo_math.h"
#include "svo_wave.h"
#include "ref_common.h"

#include <utility>

namespace svo {
#if defined(SVO_TIMELINE)
SVO_TL_DEFINE(k2v)
SVO_TL_READER(k2v)
#endif


namespace {

using namespace refsel;

constexpr int kVT = 512;              // threads per pair
constexpr int kVW = kVT / 64;         // waves
// segments of <= OW positions (a layout's one-wave size, a multiple of 256: 1024 for LayA / LayB, 512 for LayC, whose
// mailbox holds no more) continue on wave 0 (its rows 0 .. OW / 64 - 1); wave 0's register rows for the MAD pass are staged by the other waves during its one-wave rounds
// past the one-wave segment and its mailbox (mbx[2 OW, ...))
#ifndef SVO_ONEWAVE
#define SVO_ONEWAVE 2048
#endif
constexpr int kRowPad = 128;          // record planes: rows padded to two groups of 64 lanes

#include "refv_rows.h"

// A register layout: G the data registers (refv_rows.h: rows 0 .. G::kRegRows - 1 above G::kBase), R rows in all
// (the rest in LDS), a mailbox of MB doubles (Ks beyond it exchanges in chunks), PRE: the MAD pass's rows load
// during the median pass's one-wave rounds (staged in the mailbox).
template <class G, int R, uint32_t MB, bool PRE, uint32_t OW>
struct Lay {
    using Rows = G;
    static constexpr int kRows = R;
    static constexpr int kRegRows = G::kRegRows;
    static constexpr uint32_t kMbCap = MB;
    static constexpr bool kPreload = PRE;
    static constexpr uint32_t kCap = (uint32_t)R * kVT;
    static constexpr uint32_t kOneWave = OW;
    static constexpr uint32_t kStage = 2 * OW;
    static_assert(OW % 256 == 0 && OW / 64 <= G::kRegRows && OW <= 4096, "one-wave rows: register quads of wave 0");
    static_assert(R > G::kRegRows && R <= kRowPad, "rows");
    static_assert(2 * OW <= MB && MB % 64 == 0, "one-wave segment and its mailbox");
    static_assert(!PRE || kStage + 64 * G::kRegRows <= MB, "staging of wave 0's rows inside the mailbox");
    // stage_wave0: waves 1..7 take rows wave - 1 + 7 i, i < R / 7, which reaches every row only for R a multiple of 7
    static_assert(!PRE || R % (kVW - 1) == 0, "stage_wave0 covers every row");
};
#ifndef SVO_ONEWAVE_A
#define SVO_ONEWAVE_A SVO_ONEWAVE
#endif
using LayA = Lay<RowsA, 98, 12288, true, SVO_ONEWAVE_A>;   // 50 176 slots: 88 register rows (v80..v255) + 10 LDS rows
using LayB = Lay<RowsB, 118, 4352, false, SVO_ONEWAVE>;  // 60 416 slots: 92 register rows (v72..v255) + 26 LDS rows
// 65 536 slots (2621 features at patch 5): 96 register rows (v64..v255) + 32 LDS rows; the LDS rows leave a 1344-swap
// mailbox (163 032 of the CU's 163 840 LDS bytes in all), so the large rounds exchange in chunks, each walking only its
// own steps (LayC's kernels keep their compiler code below v64)
using LayC = Lay<RowsC, 128, 1344, false, 512>;
// the debug kernel (svo_debug_robust_scale: round traces, diagnostics) runs LayA / LayB with 1024-position one-wave
// rounds: its diagnostics need registers that the 2048-position one-wave code leaves below neither fence (v80 / v72).
// Both sizes run the same introselect rounds; only the point where wave 0 takes the segment over differs
using LayADbg = Lay<RowsA, 98, 12288, true, 1024>;
using LayBDbg = Lay<RowsB, 118, 4352, false, 1024>;

template <class L>
struct VShared {
    // mailbox (mbx[0, kMbCap); the one-wave segment in [0, OW) and its mailbox in [OW, 2 OW)), then the
    // per-lane dummy slots of the generic exchange rows (mbx[kMbCap + lane]): one array, so a lane's slot is
    // one selected index
    double mbx[L::kMbCap + 64];
    uint32_t rec[4][kVW][kRowPad];    // per step (row, wave) of the round: GE lo, GE hi, LE lo, LE hi masks
    uint32_t cnt[kVW][kRowPad];       // per step: #GE | #LE << 16 in it
    double pub[6];                    // pre-values published by their owners (candidates 0-3, record 4)
    uint32_t pubk[4];                 // the candidates' target ranks (0: not a target), by their owners
    double bcd;                       // broadcast of the median between the passes
    uint32_t srch[4];                 // Ks, L_{Ks+1}, R_{Ks}, L_{Ks} from wave 0
    double lrow[L::kRows - L::kRegRows][kVT];  // the LDS rows of the vector (the rest is in registers)
    uint32_t tmp[2 * kVW];            // per-wave counts of the prologue
};
static_assert(sizeof(VShared<LayC>) <= 163840, "LayC's shared state fits the CU's LDS");

struct VDiag {  // svo_debug_robust_scale diagnostics
    uint32_t nblock[2], nwave[2], heap[2], nchunk[2];
    uint64_t cyc[2];
    uint64_t ph[12];  // thread 0's cycles per phase, both passes: load, classify, barrier 1, publish + side
                      // ranks, sources, barrier 2, targets, exits (dump, one-wave rounds, final), scan, crossing,
                      // searches
    uint32_t nlog;    // (stamps build) per block round: segment size and thread 0's cycles
#if defined(SVO_STAMPS_WAVES)
    union {
        uint32_t log[64][2];
        uint32_t phw[kVW][12];  // (make stamps STAMPS_WAVES=1) every wave's cycles per phase (lane 0), in place of log
    };
#else
    uint32_t log[64][2];
#endif
    // round trace (svo_debug_robust_scale with out_len > 206; development): after every round a record of
    // kTrHead doubles (pass + 10 kind (0 block, 1 one-wave), f, l before the round, pivot, Ks, #GE, #LE, cut)
    // and the vector's M slots (a one-wave round: only its segment slots)
    double* tr;
    uint32_t trcap, ntr;
};
constexpr uint32_t kTrHead = 8;
// a phase stamp of the debug kernel in the diagnostic build (make stamps: -DSVO_STAMPS, build/stamps/); in the
// regular build the stamps are compiled out (they cost the debug kernel registers below the VGPR fence; LayB's
// debug kernel has none to spare, so it carries them in neither build)
#if defined(SVO_STAMPS_SMALL)  // (make stamps STAMPS_SMALL=1: the phases of block rounds of < 2048 positions only)
[[maybe_unused]] constexpr bool kStampsSmall = true;
#else
[[maybe_unused]] constexpr bool kStampsSmall = false;
#endif
#if defined(SVO_STAMPS) && defined(SVO_STAMPS_WAVES)
// (the wave's sums stay in scalar registers, phacc, and reach dg at the end of each pass: no memory traffic and no
// vector registers inside the rounds)
#define VSTAMP(i) \
    do { \
        if (kStampOn && dg) { \
            const uint64_t t_ = clock64(); \
            if (!kStampsSmall || small_round) phacc[i] += (uint32_t)(t_ - tstamp); \
            tstamp = t_; \
        } \
    } while (0)
#elif defined(SVO_STAMPS)
#define VSTAMP(i) \
    do { \
        if (kStampOn && dg && tid == 0) { \
            const uint64_t t_ = clock64(); \
            if (!kStampsSmall || small_round) dg->ph[i] += t_ - tstamp; \
            tstamp = t_; \
        } \
    } while (0)
#else
#define VSTAMP(i) \
    do { \
        (void)tstamp; \
    } while (0)
#endif

// The vector in registers.  Row r < G::kRegRows (positions 512 r + tid) of every lane lives in the VGPR pair
// v[B + 2r : B + 2r + 1] above the layout's fence B, outside the values the compiler allocates; the remaining rows
// live in LDS.  Every access is an asm block of refv_rows.h naming its registers (or, for a runtime row, VGPR
// indexing mode).  The compiler's own code must stay below B: tools/check_vreg_fence.py checks the generated
// assembly of every K2V kernel at every build (the Makefile fails otherwise).  Left to the compiler, the
// register-resident doubles plus the round logic did not fit 256 VGPRs: unrolled row bodies had their per-row
// values computed for all rows at once and spilled, and the VGPR-count attribute does not cap the allocation.
// the lanes of m take a, the others b: one v_cndmask on the SGPR mask (the compiler's form of
// ((m >> lane) & 1) ? a : b costs a 64-bit shift, an and and a compare per use)
__device__ __forceinline__ uint32_t lane_sel(uint64_t m, uint32_t a, uint32_t b) {
    uint32_t r;
    asm("v_cndmask_b32_e64 %0, %2, %1, %3" : "=v"(r) : "v"(a), "v"(b), "s"(m));
    return r;
}
// x with lane j (a block-uniform, dynamic lane) replaced by v: a compare and a v_cndmask (the compiler's
// v_writelane with a dynamic lane goes through M0, which the row moves overwrite)
__device__ __forceinline__ uint32_t lane_put(uint32_t x, uint32_t v, uint32_t j, uint32_t me) {
    uint32_t r;
    uint64_t eq;
    asm("v_cmp_eq_u32_e64 %1, %2, %3\n\tv_cndmask_b32_e64 %0, %4, %5, %1"
        : "=v"(r), "=&s"(eq)
        : "v"(me), "s"(j), "v"(x), "v"(v));
    return r;
}
template <class L>
struct VSel {
    using G = typename L::Rows;
    static constexpr int R = L::kRows;
    static constexpr int kVRegRows = L::kRegRows;
    static constexpr int kGenQuads = G::kGenQuads;
    static constexpr uint32_t kMbCap = L::kMbCap;
    static constexpr uint32_t kOneWave = L::kOneWave;
    static constexpr uint32_t kStage = L::kStage;
    static constexpr int kQuads = (R + 3) / 4;  // quads of rows the block rounds walk (kGenQuads of them in registers)
    // below this many rows a wave classifies and exchanges row by row (indexed registers) instead of walking the quads
#ifndef SVO_FEWROWS
#define SVO_FEWROWS 8
#endif
    static constexpr int kFewRows = SVO_FEWROWS;
    // chunked rounds walk each chunk's own steps (LayB / LayC, whose 4352- / 1344-swap mailboxes chunk the large
    // rounds; LayA's 12 288 swaps chunk none of the config-2 shape's, and the extra searches push its code past v80)
    static constexpr bool kChunkSteps = kMbCap < 12288;
#ifndef SVO_QG
#define SVO_QG 4
#endif
    static constexpr int kQG = SVO_QG;  // quads per range-tested group in the classify / exchange walks
    static constexpr bool kStampOn = L::kPreload;  // (stamps build: LayA only; LayB's registers leave no room)
    static __device__ __forceinline__ double vget(int r) { return G::vget(r); }
    static __device__ __forceinline__ void vset(int r, double x) { G::vset(r, x); }
    static __device__ __forceinline__ uint64_t vcmp_ge(int r, double p) { return G::vcmp_ge(r, p); }
    static __device__ __forceinline__ uint64_t vcmp_le(int r, double p) { return G::vcmp_le(r, p); }
    static __device__ __forceinline__ void vsel(int r, double x, uint64_t m) { G::vsel(r, x, m); }
    VShared<L>& sh;
    double* gseg;        // the pair's global scratch: the heap select's segment (depth limit only)
    uint32_t gdummy;     // its per-lane dummy slots (gseg[gdummy + lane], past every position)
    VDiag* dg;           // diagnostics (debug kernel) or nullptr
    uint32_t M, nth;
    int tid, lane, wave;
    // block-uniform selection state
    uint32_t f, l;
    uint32_t xk0 = 0, xk1 = 0;  // the exchange's current rank window (k0, k1] (a chunk's, or (0, Ks])
    int depth;
    bool rec;
    double lo_val;
    int P;
    bool small_round = false;  // (stamps build: the current block round has < 2048 positions)
#if defined(SVO_STAMPS) && defined(SVO_STAMPS_WAVES)
    uint32_t phacc[12] = {};  // (stamps build, per wave: cycles per phase of this pass so far)
#endif

    // ------------------------------------------------------------------ registers
    // body(r, x) for this wave's rows rlo..rhi, x the lane's value (kWrite: body may change it)
    template <bool kWrite, typename F>
    __device__ __forceinline__ void rows(int rlo, int rhi, F&& body) {
        const int r1 = rhi < kVRegRows - 1 ? rhi : kVRegRows - 1;
        for (int r = rlo; r <= r1; ++r) {
            double x = vget(r);
            body(r, x);
            if (kWrite) vset(r, x);
        }
#pragma unroll 2
        for (int r = rlo > kVRegRows ? rlo : kVRegRows; r <= rhi; ++r) {  // (LDS rows: 2 in flight, the registers stay low)
            double& y = sh.lrow[r - kVRegRows][tid];
            double x = y;
            body(r, x);
            if (kWrite) y = x;
        }
    }
    __device__ __forceinline__ double row_val(int r) const {
        return r < kVRegRows ? vget(r) : sh.lrow[r - kVRegRows][tid];
    }
    __device__ __forceinline__ void row_set(int r, uint32_t ln, double x) {
        if ((uint32_t)lane != ln) return;
        if (r < kVRegRows) vset(r, x);
        else sh.lrow[r - kVRegRows][tid] = x;
    }
    // this thread's rows of src: registers and LDS rows
    __device__ __forceinline__ void load_raw(const double* src) {
        constexpr int kL = R - kVRegRows;
        if constexpr (kL <= 12) {
            // the LDS rows' loads go out first and land during the register rows' loads (whose asm block ends
            // with vmcnt(0)); one latency instead of one per pair of rows
            double x[kL];
#pragma unroll
            for (int i = 0; i < kL; ++i) {
                const uint32_t q = (uint32_t)(kVRegRows + i) * kVT + (uint32_t)tid;
                x[i] = __builtin_nontemporal_load(src + (q < M ? q : 0u));
            }
            G::load(src, M * 8u, tid);  // (rows past M hold 0: never inside a segment)
#pragma unroll
            for (int i = 0; i < kL; ++i) {
                const uint32_t q = (uint32_t)(kVRegRows + i) * kVT + (uint32_t)tid;
                sh.lrow[i][tid] = q < M ? x[i] : 0.0;
            }
        } else {
            G::load(src, M * 8u, tid);
#pragma unroll 2
            for (int r = kVRegRows; r < R; ++r) {
                const uint32_t q = (uint32_t)r * kVT + (uint32_t)tid;
                sh.lrow[r - kVRegRows][tid] = q < M ? src[q] : 0.0;
            }
        }
    }
    // waves 1..7, during wave 0's one-wave rounds: wave 0's rows of src into LDS, the register rows to
    // mbx[kStage + 64 r + lane] (wave 0 moves them into its registers after the pass's last barrier: an LDS
    // latency instead of a memory latency on the critical path), the LDS rows straight into wave 0's lrow entries
    __device__ __forceinline__ void stage_wave0(const double* src) {
        double* const stg = sh.mbx + kStage;
#pragma unroll
        for (int i = 0; i < R / (kVW - 1); ++i) {
            const int r = wave - 1 + (kVW - 1) * i;
            const uint32_t q = (uint32_t)r * kVT + (uint32_t)lane;
            const double x = q < M ? src[q] : 0.0;
            if (r < kVRegRows) stg[64 * r + lane] = x;
            else sh.lrow[r - kVRegRows][lane] = x;
        }
    }
    __device__ __forceinline__ void unstage_wave0() {
        const uint32_t a = (uint32_t)(uintptr_t)(sh.mbx + kStage) + 8u * (uint32_t)lane;
        G::unstage(a);
    }
    // preloaded: the rows were loaded already (the MAD pass's rows, during the median pass's one-wave rounds)
    __device__ __forceinline__ void load(const double* src, bool mad, double med, bool preloaded) {
        if (!preloaded) load_raw(src);
        if (mad) {  // src/algorithm.cpp:860-863 (DBL_MAX stays DBL_MAX)
            const uint64_t mb = uni(__builtin_bit_cast(uint64_t, med));
            G::mad(mb);
            rows<true>(kVRegRows, R - 1, [&](int, double& x) __attribute__((always_inline)) { x = fabs(x - med); });
        }
    }
    // this wave's rows r whose step 8 r + wave lies in [s0, s1] (rlo > rhi: none)
    __device__ __forceinline__ void wave_rows(uint32_t s0, uint32_t s1, int& rlo, int& rhi) const {
        const int w = wave;
        rlo = (int)s0 <= w ? 0 : ((int)s0 - w + kVW - 1) / kVW;
        rhi = (int)s1 < w ? -1 : ((int)s1 - w) / kVW;
    }
    // lanes of this wave's step in row r inside [f, l): fw = f - 64 wave, lw = l - 64 wave
    static __device__ __forceinline__ uint64_t row_mask(int fw, int lw, int r) {
        const int b = r * kVT;
        const int lo = fw - b, hi = lw - b;
        return low_mask((uint32_t)(hi < 0 ? 0 : hi)) & ~low_mask((uint32_t)(lo < 0 ? 0 : lo));
    }
    // the owner of position q stores its current value in pub[slot]
    __device__ __forceinline__ void publish(uint32_t q, int slot) {
        if (((q >> 6) & (kVW - 1)) != (uint32_t)wave) return;
        const double x = row_val((int)(q >> 9));
        if ((uint32_t)lane == (q & 63u)) sh.pub[slot] = x;
    }
    // positions [f, l) -> dst[q - dbase]; the other lanes store to dummy + lane (branch-free)
    __device__ __forceinline__ void dump(double* dst, uint32_t dbase, double* dummy) {
        int rlo, rhi;
        wave_rows(f >> 6, (l - 1) >> 6, rlo, rhi);
        const int fo = (int)f - tid, lo = (int)l - tid;  // q = 512 r + tid in [f, l)
        double* const d = dst + ((uint32_t)tid - dbase);
        double* const dl = dummy + lane;
        rows<false>(rlo, rhi, [&](int r, double x) __attribute__((always_inline)) {
            const int b = r * kVT;
            *(b >= fo && b < lo ? d + b : dl) = x;
        });
    }

    // ------------------------------------------------------------------ 1. classification
    // This wave's rows of [f, l), in quads of four with compile-time row numbers: the two compares of a row name
    // its data registers directly (refv_rows.h), and its GE / LE masks go to lane r of four accumulators with
    // v_writelane (no per-row LDS store, no branch).  Rows outside [f, l) or partial (the first also drops
    // position f, the pivot, from GE) are masked once over the accumulators, which then go to the step records in
    // four coalesced stores per 64 rows, with the packed per-step counts the scan reads.
    struct WaveRows {
        int rlo, rhi;
        uint64_t ge_first, le_first, last;
    };
    __device__ __forceinline__ WaveRows wave_segment(uint32_t s0, uint32_t s1) const {
        WaveRows w;
        wave_rows(s0, s1, w.rlo, w.rhi);
        const int fw = (int)f - 64 * wave, lw = (int)l - 64 * wave;
        w.le_first = row_mask(fw, lw, w.rlo);
        w.last = row_mask(fw, lw, w.rhi);
        const bool own_f = ((f >> 6) & (kVW - 1)) == (uint32_t)wave && (int)(f >> 9) == w.rlo;
        w.ge_first = w.le_first & ~(own_f ? 1ull << (f & 63u) : 0ull);
        return w;
    }
    // fresh opaque copies of two uniform values: a test on them stays where it is written
    static __device__ __forceinline__ void opaque(int& a, int& b) { asm volatile("" : "+s"(a), "+s"(b)); }
    template <int Q>
    __device__ __forceinline__ void cls_quad(double p, int rlo, int rhi, uint32_t (&acc)[2][4]) {
        opaque(rlo, rhi);  // (the quad's test here, not hoisted for all quads and spilled)
        if (4 * Q + 3 < rlo || 4 * Q > rhi) return;
        cls_quad_in<Q>(p, acc);
    }
    template <int Q>
    __device__ __forceinline__ void cls_quad_in(double p, uint32_t (&acc)[2][4]) {
        constexpr int g = (4 * Q) >> 6;  // (a quad never straddles two row groups)
        if constexpr (Q < kGenQuads) {
            G::template cls4<Q>(p, acc[g]);
        } else {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int r = 4 * Q + i;
                if (r >= R) continue;
                const double x = sh.lrow[r - kVRegRows][tid];
                const uint64_t ge = __ballot(!(x < p)), le = __ballot(!(p < x));
                acc[g][0] = lane_write(acc[g][0], (uint32_t)ge, (uint32_t)(r & 63));
                acc[g][1] = lane_write(acc[g][1], (uint32_t)(ge >> 32), (uint32_t)(r & 63));
                acc[g][2] = lane_write(acc[g][2], (uint32_t)le, (uint32_t)(r & 63));
                acc[g][3] = lane_write(acc[g][3], (uint32_t)(le >> 32), (uint32_t)(r & 63));
            }
        }
    }
    // quads in groups of four (16 rows): a group outside [rlo, rhi] costs one test instead of four
    template <int Gq, int... Is>
    __device__ __forceinline__ void cls_group(double p, int rlo, int rhi, uint32_t (&acc)[2][4],
                                              std::integer_sequence<int, Is...>) {
        opaque(rlo, rhi);
        constexpr int r0 = 4 * kQG * Gq, r1 = r0 + 4 * (int)sizeof...(Is) - 1;
        if (r1 < rlo || r0 > rhi) return;
        if (r0 >= rlo && r1 <= rhi) (cls_quad_in<kQG * Gq + Is>(p, acc), ...);  // the whole group: no quad tests
        else (cls_quad<kQG * Gq + Is>(p, rlo, rhi, acc), ...);
    }
    template <int... Gs>
    __device__ __forceinline__ void cls_quads(double p, int rlo, int rhi, uint32_t (&acc)[2][4],
                                              std::integer_sequence<int, Gs...>) {
        (cls_group<Gs>(p, rlo, rhi, acc, std::make_integer_sequence<int, (kQuads - kQG * Gs < kQG ? kQuads - kQG * Gs : kQG)>{}), ...);
    }
    // a few rows: one indexed compare pair per row instead of a pass over every quad's range test
    __device__ __forceinline__ void cls_rows(double p, int rlo, int rhi, uint32_t (&acc)[2][4]) {
        for (int r = rlo; r <= rhi; ++r) {
            uint64_t ge, le;
            if (r < kVRegRows) {
                G::vcmp2(r, p, ge, le);
            } else {
                const double x = sh.lrow[r - kVRegRows][tid];
                ge = __ballot(!(x < p));
                le = __ballot(!(p < x));
            }
            // (a select per lane, not v_writelane: a runtime lane index would go through M0, which the indexed
            // row accesses overwrite)
            const bool mine = lane == (r & 63);
#pragma unroll
            for (int g = 0; g < 2; ++g) {
                if (g != (r >> 6)) continue;
                acc[g][0] = mine ? (uint32_t)ge : acc[g][0];
                acc[g][1] = mine ? (uint32_t)(ge >> 32) : acc[g][1];
                acc[g][2] = mine ? (uint32_t)le : acc[g][2];
                acc[g][3] = mine ? (uint32_t)(le >> 32) : acc[g][3];
            }
        }
    }
    __device__ __forceinline__ void classify(double p, uint32_t ch, double x0) {
        // std::iter_swap(first, chosen) of __move_median_to_first, in the owners' registers
        if (((f >> 6) & (kVW - 1)) == (uint32_t)wave) row_set((int)(f >> 9), f & 63u, p);
        if (((ch >> 6) & (kVW - 1)) == (uint32_t)wave) row_set((int)(ch >> 9), ch & 63u, x0);
        const WaveRows w = wave_segment(f >> 6, (l - 1) >> 6);
        uint32_t acc[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}};  // lane j: row 64 g + j: GE lo, GE hi, LE lo, LE hi
        if (w.rlo <= w.rhi) {
            if (w.rhi - w.rlo < kFewRows) cls_rows(p, w.rlo, w.rhi, acc);
            else cls_quads(p, w.rlo, w.rhi, acc, std::make_integer_sequence<int, (kQuads + kQG - 1) / kQG>{});
            // rows outside [rlo, rhi] (whole quads were compared) and the partial first / last rows
#pragma unroll
            for (int g = 0; g < 2; ++g) {
                const int j = 64 * g + lane;
                const bool in = j >= w.rlo && j <= w.rhi;
                uint64_t gm = in ? ~0ull : 0ull, lm = gm;
                if (j == w.rlo) { gm &= w.ge_first; lm &= w.le_first; }
                if (j == w.rhi) { gm &= w.last; lm &= w.last; }
                acc[g][0] &= (uint32_t)gm;
                acc[g][1] &= (uint32_t)(gm >> 32);
                acc[g][2] &= (uint32_t)lm;
                acc[g][3] &= (uint32_t)(lm >> 32);
            }
        }
        // the records and packed counts of all of this wave's steps (0 outside the segment)
#pragma unroll
        for (int g = 0; g < 2; ++g) {
            const int j = 64 * g + lane;
#pragma unroll
            for (int c = 0; c < 4; ++c) sh.rec[c][wave][j] = acc[g][c];
            sh.cnt[wave][j] = (__popc(acc[g][0]) + __popc(acc[g][1])) | ((__popc(acc[g][2]) + __popc(acc[g][3])) << 16);
        }
    }

    // ------------------------------------------------------------------ 2. counts, crossing, ranks (every wave)
    // Lane j holds row 64 g + j's eight packed step counts (#GE | #LE << 16, one per wave), the packed counts of all
    // steps before the row (rp) and before this wave's step of the row (pw).  A search for the last step whose
    // prefix is below a rank counts the rows whose start is below it (two ballots), then walks that row's eight
    // steps on scalars.
    struct Ctl {
        uint32_t c[2][kVW];
        uint32_t rp[2], pw[2];
        uint32_t totG, totL;
    };
    __device__ __forceinline__ void counts(Ctl& C) const {
#pragma unroll
        for (int g = 0; g < 2; ++g)
#pragma unroll
            for (int v = 0; v < kVW; ++v) C.c[g][v] = sh.cnt[v][64 * g + lane];
        uint32_t rt[2];
#pragma unroll
        for (int g = 0; g < 2; ++g) {
            uint32_t t = 0, own = 0;
#pragma unroll
            for (int v = 0; v < kVW; ++v) {
                own += v < wave ? C.c[g][v] : 0u;
                t += C.c[g][v];
            }
            rt[g] = t;
            C.pw[g] = own;
        }
        const uint32_t i0 = wave_incl_scan(rt[0]);
        const uint32_t t0 = uni(lane_read(i0, 63));
        const uint32_t i1 = wave_incl_scan(rt[1]) + t0;
        C.rp[0] = i0 - rt[0];
        C.rp[1] = i1 - rt[1];
        C.pw[0] += C.rp[0];
        C.pw[1] += C.rp[1];
        const uint32_t tot = uni(lane_read(i1, 63));
        C.totG = tot & 0xFFFFu;
        C.totL = tot >> 16;
    }
    // the packed prefix of step s (any wave's)
    template <int G>
    __device__ __forceinline__ uint32_t step_pre_g(const Ctl& C, uint32_t ln, uint32_t v) const {
        uint32_t pk = uni(lane_read(C.rp[G], (int)ln));
#pragma unroll
        for (int u = 0; u < kVW; ++u)
            if ((uint32_t)u < v) pk += uni(lane_read(C.c[G][u], (int)ln));
        return pk;
    }
    __device__ __forceinline__ uint32_t step_pre(const Ctl& C, uint32_t s) const {
        const uint32_t r = s >> 3, v = s & (kVW - 1);
        return r < 64 ? step_pre_g<0>(C, r, v) : step_pre_g<1>(C, r - 64, v);
    }
    // kind 0: #GE, 1: #LE, 2: #GE + #LE of a packed prefix
    static __device__ __forceinline__ uint32_t kval(uint32_t pk, int kind) {
        return kind == 0 ? pk & 0xFFFFu : kind == 1 ? pk >> 16 : (pk & 0xFFFFu) + (pk >> 16);
    }
    template <int G>
    __device__ __forceinline__ uint32_t walk_row(const Ctl& C, uint32_t ln, int kind, uint32_t rank, uint32_t& pre) const {
        uint32_t pk = uni(lane_read(C.rp[G], (int)ln)), s = 0, p0 = pk;
#pragma unroll
        for (int u = 0; u < kVW; ++u) {
            if (kval(pk, kind) < rank) { s = (uint32_t)u; p0 = pk; }
            pk += uni(lane_read(C.c[G][u], (int)ln));
        }
        pre = p0;
        return (64u * G + ln) * kVW + s;
    }
    // the last step whose prefix (kind) is below rank (there is one: the segment's first step has prefix 0 < rank),
    // and its packed prefix
    __device__ __forceinline__ uint32_t find_step(const Ctl& C, int kind, uint32_t rank, uint32_t& pre) const {
        const uint32_t n = popc(__ballot(kval(C.rp[0], kind) < rank)) + popc(__ballot(kval(C.rp[1], kind) < rank));
        const uint32_t jr = n - 1u;
        return jr < 64 ? walk_row<0>(C, jr, kind, rank, pre) : walk_row<1>(C, jr - 64, kind, rank, pre);
    }
    __device__ __forceinline__ uint64_t rec_mask(uint32_t s, int kind) const {
        const uint32_t r = s >> 3, v = s & (kVW - 1);
        return ((uint64_t)uni(sh.rec[2 * kind + 1][v][r]) << 32) | uni(sh.rec[2 * kind][v][r]);
    }
    // the rank-th (1-based) GE (kind 0) or LE (kind 1) position from the left
    __device__ __forceinline__ uint32_t locate(const Ctl& C, int kind, uint32_t rank) const {
        uint32_t pre;
        const uint32_t s = find_step(C, kind, rank, pre);
        return s * 64u + wave_select_bit(rec_mask(s, kind), rank - kval(pre, kind) - 1u);
    }
    // locate() reading the row's per-step counts back from LDS instead of the Ctl registers (the chunked exchange's
    // searches: the sixteen count registers would otherwise stay live through the chunk loop and push the code past
    // the VGPR fence)
    __device__ __forceinline__ uint32_t locate_lds(const Ctl& C, int kind, uint32_t rank) const {
        const uint32_t n = popc(__ballot(kval(C.rp[0], kind) < rank)) + popc(__ballot(kval(C.rp[1], kind) < rank));
        const uint32_t jr = n - 1u, g = jr >> 6, ln = jr & 63u;
        uint32_t pk = uni(lane_read(g ? C.rp[1] : C.rp[0], (int)ln)), st = 0, p0 = pk;
#pragma unroll
        for (int u = 0; u < kVW; ++u) {
            if (kval(pk, kind) < rank) { st = (uint32_t)u; p0 = pk; }
            pk += uni(sh.cnt[u][jr]);
        }
        const uint32_t s = jr * kVW + st;
        return s * 64u + wave_select_bit(rec_mask(s, kind), rank - kval(p0, kind) - 1u);
    }
    // the j-th (0-based) set bit of a uniform mask: the lane holding it has j set bits below it
    __device__ __forceinline__ uint32_t wave_select_bit(uint64_t m, uint32_t j) const {
        const uint64_t hit = __ballot(((m >> lane) & 1ull) && lanes_below(m) == j);
        return (uint32_t)__builtin_ctzll(hit);
    }
    // Ks from the crossing entry (see refsel::crossing_ks): lane b tests the split point after bit b
    __device__ __forceinline__ uint32_t wave_crossing_ks(uint32_t gcar, uint32_t lcar, uint64_t ge, uint64_t le) const {
        const uint32_t me = (uint32_t)lane;
        const uint32_t g = gcar + lanes_below(ge) + (uint32_t)((ge >> me) & 1ull);
        const uint32_t lc = lcar - (lanes_below(le) + (uint32_t)((le >> me) & 1ull));
        const uint64_t q = __ballot(g >= lc);
        const uint32_t lo = q ? (uint32_t)__builtin_ctzll(q) + 1u : 64u;  // smallest split b in [1, 64] with G >= Lc
        const uint32_t g1 = gcar + popc(ge & low_mask(lo - 1));
        const uint32_t l2 = lcar - popc(le & low_mask(lo));
        return g1 > l2 ? g1 : l2;
    }
    // candidate q of the next round (slot i): its owner publishes the pre-value and, if q is one of this round's
    // swap targets (side: 0 GE ranked from the left, 1 LE ranked from the right, rank <= ks), its rank
    __device__ __forceinline__ void publish_cand(const Ctl& C, uint32_t q, int i, uint32_t ks, int side) {
        if (((q >> 6) & (kVW - 1)) != (uint32_t)wave) return;
        const double x = row_val((int)(q >> 9));
        uint32_t k = 0;
        if (ks) {
            const uint32_t s = q >> 6, b = q & 63u, r = s >> 3;
            const uint64_t m = rec_mask(s, side);
            if ((m >> b) & 1ull) {
                const uint32_t pp = r < 64 ? uni(lane_read(C.pw[0], (int)r)) : uni(lane_read(C.pw[1], (int)(r - 64)));
                const uint32_t below = popc(m & low_mask(b));
                k = side ? C.totL - ((pp >> 16) + below) : (pp & 0xFFFFu) + below + 1u;
                if (k > ks) k = 0;
            }
        }
        if ((uint32_t)lane == (q & 63u)) {
            sh.pub[i] = x;
            sh.pubk[i] = k;
        }
    }

    // ------------------------------------------------------------------ 3. the exchange
    // side 0: GE positions ranked from the left (L_k), side 1: LE positions ranked from the right (R_k), over the
    // steps [s0, s1]; ranks k in (k0, k1]: kWrite stores the value in mb[k - 1 - k0], else the position takes it.
    // Interior rows (quads of four, refv_rows.h) recompute the side's mask from the registers, select the lanes
    // that take part through EXEC and need no rank test: every rank there lies inside (k0, k1] when the round has
    // one chunk (the one rank boundary, at L_Ks / R_Ks, lies in step bstep, whose row goes the generic way).  The
    // wave's first and last rows (partial at the segment's ends), that row, the LDS rows and every row of a chunked
    // round take the generic path (masks with the range test; a chunked round takes the masks from the records,
    // since an earlier chunk's targets may have changed registers a recompute would read).
    template <bool kWrite>
    __device__ __forceinline__ void generic_row(const Ctl& C, int side, int r, uint64_t gm, double p, uint32_t k0,
                                                uint32_t k1, bool chunked) {
        const uint32_t pp = r < 64 ? uni(lane_read(C.pw[0], r)) : uni(lane_read(C.pw[1], r - 64));
        const uint32_t nk = k1 - k0;
        const uint32_t b = side == 0 ? (pp & 0xFFFFu) - k0 : C.totL - 1u - k0 - (pp >> 16);
        double* const mbx = sh.mbx;
        const uint32_t dslot = kMbCap + (uint32_t)lane;
        uint64_t m;
        double x = 0.0;
        const bool reg = r < kVRegRows;
        if (!reg) x = sh.lrow[r - kVRegRows][tid];
        if (chunked) m = rec_mask((uint32_t)(r * kVW + wave), side);
        else if (side == 0) m = reg ? vcmp_ge(r, p) : __ballot(!(x < p));
        else m = reg ? vcmp_le(r, p) : __ballot(!(p < x));
        m &= gm;
        const uint32_t kk = side == 0 ? b + lanes_below(m) : b - lanes_below(m);
        const uint64_t okm = m & __ballot(kk < nk);
        const uint32_t a = lane_sel(okm, kk, dslot);
        if (kWrite) {
            mbx[a] = reg ? vget(r) : x;
        } else {
            const double t = mbx[a];
            if (reg) vsel(r, t, okm);
            else if ((okm >> lane) & 1ull) sh.lrow[r - kVRegRows][tid] = t;
        }
    }
    // rows ra..rb of this wave; pb[g]: lane j the mailbox byte address of row 64 g + j's slot 0 (of the chunk's ranks
    // (xk0, xk1], which the LDS rows' generic path tests)
    template <int Q, bool kWrite, int S>
    __device__ __forceinline__ void ex_quad(const Ctl& C, double p, int ra, int rb, const uint32_t (&pb)[2]) {
        opaque(ra, rb);
        if (4 * Q + 3 < ra || 4 * Q > rb) return;
        constexpr int g = (4 * Q) >> 6;
        if constexpr (Q < kGenQuads) {
            if (4 * Q >= ra && 4 * Q + 3 <= rb) {  // interior quad: all four rows
                if (kWrite) G::template src4<Q, S>(p, pb[g]);
                else G::template tgt4<Q, S>(p, pb[g]);
            } else {
                if (kWrite) G::template src4e<Q, S>(p, pb[g], (uint32_t)ra, (uint32_t)(rb - ra));
                else G::template tgt4e<Q, S>(p, pb[g], (uint32_t)ra, (uint32_t)(rb - ra));
            }
        } else {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int r = 4 * Q + i;
                if (r < R && r >= ra && r <= rb) generic_row<kWrite>(C, S, r, ~0ull, p, xk0, xk1, false);
            }
        }
    }
    // a quad wholly inside the range: every row takes part, no test
    template <int Q, bool kWrite, int S>
    __device__ __forceinline__ void ex_quad_in(const Ctl& C, double p, const uint32_t (&pb)[2]) {
        constexpr int g = (4 * Q) >> 6;
        if constexpr (Q < kGenQuads) {
            if (kWrite) G::template src4<Q, S>(p, pb[g]);
            else G::template tgt4<Q, S>(p, pb[g]);
        } else {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int r = 4 * Q + i;
                if (r < R) generic_row<kWrite>(C, S, r, ~0ull, p, xk0, xk1, false);
            }
        }
    }
    template <bool kWrite, int S>
    __device__ __forceinline__ void ex_quads(const Ctl& C, double p, int ra, int rb, uint32_t k0) {
        const uint32_t mb = (uint32_t)(uintptr_t)sh.mbx - 8u * k0;  // (a chunk's ranks (k0, k1] in slots 0 ..)
        uint32_t pb[2];
#pragma unroll
        for (int g = 0; g < 2; ++g)
            pb[g] = S == 0 ? mb + 8u * (C.pw[g] & 0xFFFFu) : mb + 8u * (C.totL - 1u - (C.pw[g] >> 16));
        ex_groups<kWrite, S>(C, p, ra, rb, pb, std::make_integer_sequence<int, (kQuads + kQG - 1) / kQG>{});
    }
    template <bool kWrite, int S, int Gq, int... Is>
    __device__ __forceinline__ void ex_group(const Ctl& C, double p, int ra, int rb, const uint32_t (&pb)[2],
                                             std::integer_sequence<int, Is...>) {
        opaque(ra, rb);
        constexpr int r0 = 4 * kQG * Gq, r1 = r0 + 4 * (int)sizeof...(Is) - 1;
        if (r1 < ra || r0 > rb) return;
        if (r0 >= ra && r1 <= rb) {  // whole group inside
            if constexpr (!kWrite && G::kTgt8 && kQG == 4 && sizeof...(Is) == 4 && r1 < 4 * kGenQuads) {
                G::template tgt8<2 * Gq, S>(p, pb[r0 >> 6]);  // (eight mailbox reads in flight per block)
                G::template tgt8<2 * Gq + 1, S>(p, pb[r0 >> 6]);
            } else {
                (ex_quad_in<kQG * Gq + Is, kWrite, S>(C, p, pb), ...);
            }
        }
        else (ex_quad<kQG * Gq + Is, kWrite, S>(C, p, ra, rb, pb), ...);
    }
    template <bool kWrite, int S, int... Gs>
    __device__ __forceinline__ void ex_groups(const Ctl& C, double p, int ra, int rb, const uint32_t (&pb)[2],
                                              std::integer_sequence<int, Gs...>) {
        (ex_group<kWrite, S, Gs>(C, p, ra, rb, pb,
                                 std::make_integer_sequence<int, (kQuads - kQG * Gs < kQG ? kQuads - kQG * Gs : kQG)>{}), ...);
    }
    template <bool kWrite>
    __device__ __forceinline__ void exchange(const Ctl& C, int side, uint32_t s0, uint32_t s1, uint32_t bstep, double p,
                                             uint32_t k0, uint32_t k1, bool chunked) {
        // (fresh opaque copies: the compiler would otherwise compute both sides' row ranges and masks for the sources
        // and the targets up front and keep them, spilled, across the barrier)
        asm volatile("" : "+s"(s0), "+s"(s1));
        const WaveRows w = wave_segment(s0, s1);
        if (w.rlo > w.rhi) return;
        const uint64_t gfirst = side == 0 ? w.ge_first : w.le_first;
        if (chunked && !kChunkSteps) {  // (LayA: never for the config-2 shape) every row generic, masks from the records
            for (int r = w.rlo; r <= w.rhi; ++r)
                generic_row<kWrite>(C, side, r, r == w.rlo ? gfirst : (r == w.rhi ? w.last : ~0ull), p, k0, k1, true);
            return;
        }
        // (a chunk's end rows take their masks from the records: an earlier chunk's targets may sit in its first or
        // last step; every step between holds only this chunk's ranks and rows no earlier chunk touched)
        generic_row<kWrite>(C, side, w.rlo, w.rlo == w.rhi ? gfirst & w.last : gfirst, p, k0, k1, chunked);
        if (w.rhi > w.rlo) generic_row<kWrite>(C, side, w.rhi, w.last, p, k0, k1, chunked);
        // (the rank boundaries (L_Ks / R_Ks, or a chunk's first and last ranks) lie in the first / last step of the
        // range, so their rows are end rows of the waves that own those steps: the interior rows need no rank test)
        (void)bstep;
        const int ra = w.rlo + 1, rb = w.rhi - 1;
        if (ra > rb) return;
        if (rb - ra < kFewRows) {  // a few rows: the generic way, no pass over every quad's range test
            for (int r = ra; r <= rb; ++r) generic_row<kWrite>(C, side, r, ~0ull, p, k0, k1, false);
            return;
        }
        xk0 = k0;
        xk1 = k1;
        if (side == 0) ex_quads<kWrite, 0>(C, p, ra, rb, k0);
        else ex_quads<kWrite, 1>(C, p, ra, rb, k0);
    }

    // ------------------------------------------------------------------ one block round
    // pivot p (moved to f), x0 the value moved to ch; on return [f, l) is the kept side and cand[] the next
    // round's A, B, C, first values (when another block round follows)
    // fresh opaque copies of the thread / lane / wave numbers: values derived from them would otherwise be
    // hoisted out of the round loop and held in registers for all of it
    __device__ __forceinline__ void refresh_ids() {
        asm volatile("" : "+v"(tid), "+v"(lane));
        wave = (int)uni((uint32_t)tid >> 6);
    }
    // the round trace (debug kernel only: dg->tr set; compiled out of the stamps build, whose clock reads need the
    // registers the trace code holds)
    __device__ __forceinline__ bool tracing() const {
#if defined(SVO_STAMPS)
        return false;
#else
        return dg && dg->tr;
#endif
    }
    __device__ __forceinline__ double* trace_rec(uint32_t kind, uint32_t f0, uint32_t l0, double p, uint32_t ks,
                                                 uint32_t tg, uint32_t tl, uint32_t cut) {
        if (!tracing()) return nullptr;
        const uint32_t i = dg->ntr;
        if ((uint64_t)(i + 1u) * (kTrHead + M) > dg->trcap) return nullptr;
        double* const b = dg->tr + (uint64_t)i * (kTrHead + M);
        // one header field per lane of threads 0..7 (wave 0): a register pair, not the whole header, stays live
        if (tid < (int)kTrHead) {
            const uint32_t j = (uint32_t)tid;
            const uint32_t u = j == 0 ? (uint32_t)(P + 10 * (int)kind) : j == 1 ? f0 : j == 2 ? l0 : j == 4 ? ks
                             : j == 5 ? tg : j == 6 ? tl : cut;
            b[j] = j == 3 ? p : (double)u;
        }
        return b + kTrHead;
    }
    __device__ __forceinline__ void trace_block(uint32_t f0, uint32_t l0, double p, uint32_t ks, uint32_t tg, uint32_t tl,
                                                uint32_t cut) {
        double* const v = trace_rec(0, f0, l0, p, ks, tg, tl, cut);
        if (v) {
            rows<false>(0, R - 1, [&](int r, double x) __attribute__((always_inline)) {
                const uint32_t q = (uint32_t)r * kVT + (uint32_t)tid;
                if (q < M) v[q] = x;
            });
        }
        __syncthreads();
        if (tracing() && tid == 0) ++dg->ntr;
        __syncthreads();
    }
    __device__ __forceinline__ void block_round(double p, uint32_t ch, double x0, double (&cand)[4]) {
        refresh_ids();
        uint64_t tstamp = dg ? clock64() : 0;
#if defined(SVO_STAMPS)
        const uint64_t tround = tstamp;
        const uint32_t S0 = l - f;
        small_round = S0 < 2048;
#endif
        classify(p, ch, x0);
        VSTAMP(1);
        __syncthreads();
        VSTAMP(2);
        Ctl C;
        counts(C);
        VSTAMP(8);
        const uint32_t totL = C.totL, totG = C.totG;
        uint32_t ks, lk1, rk, lk;
        // which of L_{Ks+1}, R_{Ks}, L_{Ks} to find (bits 0, 1, 2)
        auto search = [&](int which) __attribute__((always_inline)) {
            // the crossing: the last step whose start has G < Lc, i.e. G + L < totL (the segment's first step always)
            uint32_t pke;
            const uint32_t es = find_step(C, 2, totL, pke);
            const uint64_t mge = rec_mask(es, 0), mle = rec_mask(es, 1);
            ks = uni(wave_crossing_ks(pke & 0xFFFFu, totL - (pke >> 16), mge, mle));
            VSTAMP(9);
            // L_{Ks+1} (GE rank Ks + 1), R_{Ks} (LE rank totL - Ks + 1 from the left), L_{Ks}: all three sit next to
            // the crossing split, so they are looked for in the crossing step first
            const uint32_t ra = ks + 1u, rb = totL - ks + 1u, rc = ks;
            const uint32_t G0 = pke & 0xFFFFu, L0 = pke >> 16, cg = popc(mge), cl = popc(mle);
            const uint32_t ebase = es * 64u;
            if (which & 1)
                lk1 = ra > totG ? kNone
                      : (ra > G0 && ra <= G0 + cg) ? ebase + uni(wave_select_bit(mge, ra - G0 - 1u)) : uni(locate(C, 0, ra));
            if (which & 2)
                rk = ks == 0 ? kNone
                     : (rb > L0 && rb <= L0 + cl) ? ebase + uni(wave_select_bit(mle, rb - L0 - 1u)) : uni(locate(C, 1, rb));
            if (which & 4)
                lk = ks == 0 ? kNone
                     : (rc > G0 && rc <= G0 + cg) ? ebase + uni(wave_select_bit(mge, rc - G0 - 1u)) : uni(locate(C, 0, rc));
            VSTAMP(10);
        };
#if defined(SVO_K2V_ONECHAIN)
        // the scalar search chain once, on wave 0 (the oldest wave, first in issue); the others wait at a barrier
        // instead of running seven more copies of it beside their SIMD partners, then read the four results
        // (round 5, same box A/B: 165.6k -> 166.9k pairs/s alone, 168.7k -> 170.2k on top of the ILP quads)
        if (wave == 0) {
            search(7);
            if (lane == 0) {
                sh.srch[0] = ks;
                sh.srch[1] = lk1;
                sh.srch[2] = rk;
                sh.srch[3] = lk;
            }
        }
        __syncthreads();
        ks = uni(sh.srch[0]);
        lk1 = uni(sh.srch[1]);
        rk = uni(sh.srch[2]);
        lk = uni(sh.srch[3]);
#elif !defined(SVO_K2V_ALLCHAINS)
        // the three boundary searches side by side on waves 0, 1, 2 (three SIMDs), each after its own copy of the
        // crossing search; the other waves wait at the barrier (round 5, same box: 170.1k -> 172.7k pairs/s over
        // -DSVO_K2V_ONECHAIN, all three on wave 0; -DSVO_K2V_ALLCHAINS: round 4's every-wave form)
        if (wave < 3) {
            search(1 << wave);
            if (lane == 0) {
                if (wave == 0) {
                    sh.srch[0] = ks;
                    sh.srch[1] = lk1;
                } else if (wave == 1) {
                    sh.srch[2] = rk;
                } else {
                    sh.srch[3] = lk;
                }
            }
        }
        __syncthreads();
        ks = uni(sh.srch[0]);
        lk1 = uni(sh.srch[1]);
        rk = uni(sh.srch[2]);
        lk = uni(sh.srch[3]);
#else
        search(7);
#endif
        const uint32_t cut = lk1 < rk ? lk1 : rk;
        const bool right = cut <= nth;  // the side introselect continues with
        const uint32_t nf = right ? cut : f, nl = right ? l : cut;
        // vec[nth - 1] after this round (never touched again): only L_{Ks} can sit at cut - 1
        const bool record = cut == nth && !rec;
        if (record) publish(lk == cut - 1u ? rk : cut - 1u, 4);
        const uint32_t nS = nl - nf;
        const bool need = nS > kOneWave && depth > 0;  // another block round follows
        const uint32_t cq[4] = {nf + 1u, nf + nS / 2u, nl - 1u, nf};
        // sources: the side the kept side takes its values from; targets: the kept side's swapped positions
        const int src_side = right ? 0 : 1, tgt_side = right ? 1 : 0;
        if (need) {
#pragma unroll
            for (int i = 0; i < 4; ++i) publish_cand(C, cq[i], i, ks, tgt_side);
        }
        const uint32_t sl = (l - 1) >> 6;
        const uint32_t s0L = f >> 6, s1L = lk != kNone ? lk >> 6 : 0u;       // L_k, k <= Ks (boundary: s1L)
        const uint32_t s0R = rk != kNone ? rk >> 6 : sl + 1u, s1R = sl;       // R_k, k <= Ks (boundary: s0R)
        // Ks beyond the mailbox: chunks of kMbCap ranks, the masks from the records (see exchange).
        const uint32_t nch = ks == 0 ? 1u : (ks + kMbCap - 1u) / kMbCap;
        uint32_t ck[4] = {0, 0, 0, 0};  // the candidates' target ranks (0: not a target)
        VSTAMP(3);
        // a chunk's steps on one side: the positions of its ranks (k0, k1] (side 0: GE ranked from the left, L_k;
        // side 1: LE ranked from the right, R_k) are contiguous, so a chunk walks only the steps from its first to its
        // last rank's instead of the side's whole range (a chunked round then visits each row about once, not nch times)
        auto chunk_steps = [&](int side, uint32_t k0, uint32_t k1, uint32_t& s0, uint32_t& s1) __attribute__((always_inline)) {
            if (side == 0) {
                s0 = uni(locate_lds(C, 0, k0 + 1u)) >> 6;
                s1 = uni(locate_lds(C, 0, k1)) >> 6;
            } else {
                s0 = uni(locate_lds(C, 1, C.totL - k1 + 1u)) >> 6;
                s1 = uni(locate_lds(C, 1, C.totL - k0)) >> 6;
            }
        };
        for (uint32_t it = 0; it < nch; ++it) {
            const uint32_t k0 = it * kMbCap, k1 = ks < k0 + kMbCap ? ks : k0 + kMbCap;
            if (ks) {
                if (kChunkSteps && nch > 1) {
                    uint32_t c0, c1;
                    chunk_steps(src_side, k0, k1, c0, c1);
                    if (src_side == 0) exchange<true>(C, 0, c0, c1, c1, p, k0, k1, true);
                    else exchange<true>(C, 1, c0, c1, c0, p, k0, k1, true);
                } else if (src_side == 0) {
                    exchange<true>(C, 0, s0L, s1L, s1L, p, k0, k1, nch > 1);
                } else {
                    exchange<true>(C, 1, s0R, s1R, s0R, p, k0, k1, nch > 1);
                }
            }
            VSTAMP(4);
            __syncthreads();
            VSTAMP(5);
            if (it == 0) {
                if (record) { lo_val = uni(sh.pub[4]); rec = true; }
                if (need) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        cand[i] = uni(sh.pub[i]);
                        ck[i] = uni(sh.pubk[i]);
                    }
                }
            }
            if (ks) {
                if (kChunkSteps && nch > 1) {
                    uint32_t c0, c1;
                    chunk_steps(tgt_side, k0, k1, c0, c1);
                    if (tgt_side == 0) exchange<false>(C, 0, c0, c1, c1, p, k0, k1, true);
                    else exchange<false>(C, 1, c0, c1, c0, p, k0, k1, true);
                } else if (tgt_side == 0) {
                    exchange<false>(C, 0, s0L, s1L, s1L, p, k0, k1, nch > 1);
                } else {
                    exchange<false>(C, 1, s0R, s1R, s0R, p, k0, k1, nch > 1);
                }
                if (need) {
#pragma unroll
                    for (int i = 0; i < 4; ++i)
                        if (ck[i] > k0 && ck[i] <= k1) cand[i] = uni(sh.mbx[ck[i] - 1u - k0]);
                }
            }
            if (it + 1 < nch) __syncthreads();
        }
        if (nch > 1) __syncthreads();  // (records read above until here)
        VSTAMP(6);
        if (dg && tid == 0) dg->nchunk[P] += nch > 1 ? 1u : 0u;
#if defined(SVO_STAMPS) && !defined(SVO_STAMPS_WAVES)
        if (kStampOn && dg && tid == 0 && dg->nlog < 64) {
            dg->log[dg->nlog][0] = S0;
            dg->log[dg->nlog][1] = (uint32_t)(clock64() - tround);
            ++dg->nlog;
        }
#endif
        if (tracing()) {
            const uint32_t f0 = f, l0 = l;
            f = nf;
            l = nl;
            trace_block(f0, l0, p, ks, totG, totL, cut);
        }
        f = nf;
        l = nl;
    }

    // ------------------------------------------------------------------ rounds of <= 512 positions (wave 0)
    // No barriers: wave 0 takes the segment (seg[i] = position f0 + i, from the dump) into its data rows 0 .. OW / 64 - 1
    // (position f0 + 64 j + L in lane L of row j; the rows' own values are dead after the dump), so a round
    // reads no segment memory: the candidates are readlanes; the classification is cls4's compares with the masks
    // in lane j of four accumulators (row j = lane j), the packed counts and their prefixes one DPP scan, the
    // crossing and the rank searches ballots over the row lanes; the swaps go through the mailbox mb (a wave's LDS
    // accesses complete in program order) by w1src / w1tgt (refv_rows.h).  Stops at <= 3 positions or depth 0;
    // then the rows go back to seg for the final sort or the heap select.
    __device__ __forceinline__ double cand_at(uint32_t q) const {
        return uni(lane_read(vget((int)(q >> 6)), (int)(q & 63u)));
    }
    // the one-wave round's quads of rows (Q = 0 .. kOneWave / 256 - 1) that meet rows [js, je]
    template <int Q>
    static __device__ __forceinline__ void w1_cls(double pe, uint32_t (&acc)[4], int js, int je) {
        if constexpr (Q < (int)(kOneWave / 256)) {
            if (js <= 4 * Q + 3 && je >= 4 * Q) G::template cls4<Q>(pe, acc);
            w1_cls<Q + 1>(pe, acc, js, je);
        }
    }
    template <int Q, int S, bool W>
    static __device__ __forceinline__ void w1_ex(uint32_t ml, uint32_t mh, uint32_t pkv, uint32_t ks, uint32_t tl1,
                                                 uint32_t mbb, int js, int je) {
        if constexpr (Q < (int)(kOneWave / 256)) {
            if (js <= 4 * Q + 3 && je >= 4 * Q) {
                if constexpr (W) G::template w1src<Q, S>(ml, mh, pkv, ks, tl1, mbb);
                else G::template w1tgt<Q, S>(ml, mh, pkv, ks, tl1, mbb);
            }
            w1_ex<Q + 1, S, W>(ml, mh, pkv, ks, tl1, mbb, js, je);
        }
    }
    __device__ __forceinline__ void wave_rounds(double* seg, double* mb, uint32_t& nrounds) {
        const uint32_t f0 = f, me = (uint32_t)lane;
        uint32_t fr = 0, lr = l - f;
        const uint32_t nrel = nth - f0;
#pragma unroll
        for (int j = 0; j < (int)(kOneWave / 64); ++j) vset(j, seg[64 * j + lane]);
        const uint32_t mbb = (uint32_t)(uintptr_t)mb;
        while (lr - fr > 64 && depth > 0) {  // (<= 64 positions: the one-row rounds below)
            --depth;
            ++nrounds;
            const uint32_t A = fr + 1, B = fr + (lr - fr) / 2, C = lr - 1;
            const double a = cand_at(A), b = cand_at(B), c = cand_at(C), xv = cand_at(fr);
            uint32_t chh;
            double pe;
            median3(a, b, c, A, B, C, chh, pe);
            // std::iter_swap(first, chosen)
            vsel((int)(fr >> 6), pe, 1ull << (fr & 63u));
            vsel((int)(chh >> 6), xv, 1ull << (chh & 63u));
            int js = (int)(fr >> 6), je = (int)((lr - 1) >> 6);
            uint32_t acc[4] = {0, 0, 0, 0};  // lane j: row j's GE lo, GE hi, LE lo, LE hi
            opaque(js, je);
            w1_cls<0>(pe, acc, js, je);
            // the rows' parts inside [fr, lr) (GE without the pivot at fr)
            const bool live = (int)me >= js && (int)me <= je;
            const uint32_t rb0 = 64u * me;
            const uint32_t lo = fr > rb0 ? fr - rb0 : 0u;
            const uint32_t hi = live ? (lr - rb0 < 64u ? lr - rb0 : 64u) : 0u;
            const uint64_t inm = live ? low_mask(hi) & ~low_mask(lo) : 0ull;
            const uint64_t gem = inm & ~((int)me == js ? 1ull << (fr & 63u) : 0ull);
            acc[0] &= (uint32_t)gem;
            acc[1] &= (uint32_t)(gem >> 32);
            acc[2] &= (uint32_t)inm;
            acc[3] &= (uint32_t)(inm >> 32);
            const uint32_t cnt = ((uint32_t)__popc(acc[0]) + (uint32_t)__popc(acc[1])) |
                                 (((uint32_t)__popc(acc[2]) + (uint32_t)__popc(acc[3])) << 16);
            const uint32_t incl = wave_incl_scan(cnt);
            const uint32_t pkv = incl - cnt;  // lane j: #GE | #LE << 16 before row j
            const uint32_t tot = uni(lane_read(incl, 63));
            const uint32_t tG = tot & 0xFFFFu, tL = tot >> 16;
            const uint32_t gpl = pkv & 0xFFFFu, lpl = pkv >> 16;
            auto masks = [&](uint32_t jj, uint64_t& ge, uint64_t& le) __attribute__((always_inline)) {
                ge = ((uint64_t)uni(lane_read(acc[1], (int)jj)) << 32) | uni(lane_read(acc[0], (int)jj));
                le = ((uint64_t)uni(lane_read(acc[3], (int)jj)) << 32) | uni(lane_read(acc[2], (int)jj));
            };
            // crossing: the last live row whose start has G < Lc, i.e. G + L < tL (row js always)
            const uint64_t cq = __ballot(live && gpl + lpl < tL);
            const uint32_t jc = 63u - (uint32_t)__builtin_clzll(cq);
            uint64_t a0, b0m;
            masks(jc, a0, b0m);
            const uint32_t pkc = uni(lane_read(pkv, (int)jc));
            const uint32_t ks = uni(wave_crossing_ks(pkc & 0xFFFFu, tL - (pkc >> 16), a0, b0m));
            // the rank-th GE (kind 0) / LE (kind 1) position: the last live row starting below the rank
            auto rank_pos = [&](int kind, uint32_t rank) __attribute__((always_inline)) -> uint32_t {
                if (rank == 0 || rank > (kind ? tL : tG)) return kNone;
                const uint64_t q = __ballot(live && (kind ? lpl : gpl) < rank);
                const uint32_t jj = 63u - (uint32_t)__builtin_clzll(q);
                const uint32_t pp = uni(lane_read(pkv, (int)jj));
                const uint32_t pre = kind ? pp >> 16 : pp & 0xFFFFu;
                uint64_t ge, le;
                masks(jj, ge, le);
                return 64u * jj + wave_select_bit(kind ? le : ge, rank - pre - 1u);
            };
            const uint32_t lk1 = rank_pos(0, ks + 1), rk = ks >= 1 ? rank_pos(1, tL - ks + 1) : kNone;
            const uint32_t cut = lk1 < rk ? lk1 : rk;
            const bool right = cut <= nrel;
            if (cut == nrel && !rec && nrel >= 1) {
                const uint32_t lk = ks >= 1 ? rank_pos(0, ks) : kNone;
                lo_val = cand_at(lk == cut - 1 ? rk : cut - 1);  // (pre-values: the swaps come below)
                rec = true;
            }
            // sources to the mailbox, then the kept side's targets take it (rows js..je: empty rows have no lanes)
            if (ks) {
                const uint32_t tl1 = tL - 1u;
                // L_k (k <= Ks) all lie below the cut and R_k (k <= Ks) at or above it: each side walks only its rows
                const int jl = (int)((cut - 1u) >> 6), jr = (int)(cut >> 6);
                if (right) {
                    w1_ex<0, 0, true>(acc[0], acc[1], pkv, ks, tl1, mbb, js, jl);
                    w1_ex<0, 1, false>(acc[2], acc[3], pkv, ks, tl1, mbb, jr, je);
                } else {
                    w1_ex<0, 1, true>(acc[2], acc[3], pkv, ks, tl1, mbb, jr, je);
                    w1_ex<0, 0, false>(acc[0], acc[1], pkv, ks, tl1, mbb, js, jl);
                }
            }
            if (tracing()) {  // (wave 0 only: no barrier; the record counter is wave 0's)
                double* const v = trace_rec(1, f0 + fr, f0 + lr, pe, ks, tG, tL, f0 + cut);
                if (v) {
#pragma unroll
                    for (int j = 0; j < (int)(kOneWave / 64); ++j)
                        if (f0 + 64u * j + me < M) v[f0 + 64u * j + me] = vget(j);
                    if (me == 0) ++dg->ntr;
                }
            }
            if (right) fr = cut;
            else lr = cut;
        }
#pragma unroll
        for (int j = 0; j < (int)(kOneWave / 64); ++j) seg[64 * j + lane] = vget(j);
        if (lr - fr > 3 && depth > 0) row_rounds(seg, reinterpret_cast<uint32_t*>(mb), f0, fr, lr, nrounds);
        f = f0 + fr;
        l = f0 + lr;
    }
    // Rounds of <= 64 positions on one register pair (wave 0): lane i holds position f0 + w + i (w = fr at entry)
    // and [a, b) is the segment in lanes.  Masks are ballots, ranks mbcnt, Ks the crossing over the 64 split
    // points, and the swaps L_k <-> R_k one lane permutation: each swapping lane finds its partner's lane in a
    // 64-entry table in the mailbox (written by the partners, read by the same wave in program order) and takes
    // its value by ds_bpermute.  No position is both a swapping GE and a swapping LE (L_k < R_k for k <= Ks), so
    // every lane has at most one partner.  Then the lanes go back to seg.
    __device__ __forceinline__ void row_rounds(double* seg, uint32_t* tab, uint32_t f0, uint32_t& fr, uint32_t& lr,
                                               uint32_t& nrounds) {
        const uint32_t me = (uint32_t)lane, w = fr, n0 = lr - fr;
        const uint32_t nr = nth - f0 - w;  // nth in lanes (inside [0, n0))
        double x = seg[w + me];            // (lanes past n0 read the slots after: never live)
        uint32_t a = 0, b = n0;
        while (b - a > 3 && depth > 0) {
            --depth;
            ++nrounds;
            const uint32_t A = a + 1, B = a + (b - a) / 2, C = b - 1;
            const double va = uni(lane_read(x, (int)A)), vb = uni(lane_read(x, (int)B)), vc = uni(lane_read(x, (int)C));
            const double x0 = uni(lane_read(x, (int)a));
            uint32_t ch;
            double pe;
            median3(va, vb, vc, A, B, C, ch, pe);
            x = me == a ? pe : (me == ch ? x0 : x);  // std::iter_swap(first, chosen)
            const bool live = me >= a && me < b;
            const uint64_t ge = __ballot(live && me != a && !(x < pe)), le = __ballot(live && !(pe < x));
            const uint32_t tG = popc(ge), tL = popc(le);
            const uint32_t ks = uni(wave_crossing_ks(0u, tL, ge, le));
            const uint32_t lk1 = ks + 1u <= tG ? uni(wave_select_bit(ge, ks)) : kNone;
            const uint32_t rk = ks >= 1u ? uni(wave_select_bit(le, tL - ks)) : kNone;
            const uint32_t cut = lk1 < rk ? lk1 : rk;
            if (cut == nr && !rec && nth >= 1u) {  // vec[nth - 1] after this round (pre-swap values, see block_round)
                const uint32_t lk = ks >= 1u ? uni(wave_select_bit(ge, ks - 1u)) : kNone;
                lo_val = uni(lane_read(x, (int)(lk == cut - 1u ? rk : cut - 1u)));
                rec = true;
            }
            if (ks) {
                // GE rank k (from the left) <-> LE rank k (from the right), k <= Ks
                const uint32_t kg = lanes_below(ge) + 1u, kl = tL - lanes_below(le);
                const bool sg = ((ge >> me) & 1ull) && kg <= ks, sl = ((le >> me) & 1ull) && kl <= ks;
                if (sl) tab[kl - 1u] = me;
                if (sg) tab[64u + kg - 1u] = me;
                // (the table entries come from other lanes: a compiler memory barrier keeps the loads after the
                // stores; the LDS keeps one wave's accesses in order)
                asm volatile("" ::: "memory");
                const uint32_t partner = sg ? tab[kg - 1u] : (sl ? tab[64u + kl - 1u] : me);
                const uint64_t u = __builtin_bit_cast(uint64_t, x);
                const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(partner * 4u), (int)(uint32_t)u);
                const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(partner * 4u), (int)(uint32_t)(u >> 32));
                x = __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
                asm volatile("" ::: "memory");
            }
            if (tracing()) {
                double* const v = trace_rec(1, f0 + w + a, f0 + w + b, pe, ks, tG, tL, f0 + w + cut);
                if (v) {
                    if (me < n0) v[f0 + w + me] = x;
                    if (me == 0) ++dg->ntr;
                }
            }
            if (cut <= nr) a = cut;
            else b = cut;
        }
        if (me < n0) seg[w + me] = x;
        fr = w + a;
        lr = w + b;
    }
    // ------------------------------------------------------------------ std::nth_element(vec, vec + nth)
    // (vec[nth - 1], vec[nth]) of the post-state, on thread 0
    // preload_next: load the raw rows for the MAD pass while wave 0 runs this pass's one-wave rounds (the other
    // waves' registers are free after the dump); returns through `preloaded` whether it did
    // retire (the last pass): once the segment has gone to wave 0's one-wave rounds, waves 1-7 end here instead of
    // waiting at the pass's remaining barriers; an ended wave frees its SIMD's registers for other kernels' workgroups
    // and no longer counts at s_barrier.  `retired` tells the caller to return.
    __device__ __forceinline__ void select(const double* src, bool mad, double med, bool preloaded, bool preload_next,
                                           double& hi, double& lo, bool& did_preload, bool retire, bool& retired) {
        const uint64_t t0 = dg ? clock64() : 0;
        uint64_t tstamp = t0;
        did_preload = false;
        load(src, mad, med, preloaded);
        VSTAMP(0);
        f = 0;
        l = M;
        depth = M > 1 ? 2 * lg2(M) : 0;
        rec = false;
        lo_val = 0.0;
        double cand[4] = {0.0, 0.0, 0.0, 0.0};
        if (M >= 4) {  // round 1's candidates straight from the source (uniform loads)
            const uint32_t qs[4] = {1u, M / 2u, M - 1u, 0u};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const double x = src[qs[i]];
                cand[i] = uni(mad ? fabs(x - med) : x);
            }
        }
        uint32_t nblock = 0;
        while (l - f > kOneWave && depth > 0) {
            --depth;
            ++nblock;
            uint32_t ch;
            double p;
            median3(cand[0], cand[1], cand[2], f + 1u, f + (l - f) / 2u, l - 1u, ch, p);
            block_round(uni(p), uni(ch), cand[3], cand);
        }
        tstamp = dg ? clock64() : 0;
        __syncthreads();  // the last round's targets still read the mailbox the exits overwrite
        if (l - f > kOneWave) {  // depth limit on a large segment: heap select in the pair's global scratch
            dump(gseg, 0, gseg + gdummy);
            __threadfence_block();
            __syncthreads();
            if (tid == 0) {
                heap_select_at(gseg + f, l - f, nth + 1 - f, nth - f);
                hi = gseg[nth];
                lo = rec ? lo_val : (nth >= 1 ? gseg[nth - 1] : 0.0);
            }
            if (dg && tid == 0) dg->heap[P] = 1;
        } else {
            double* const seg = sh.mbx;  // positions f0 + i
            const uint32_t f0 = f;
            dump(seg, f0, sh.mbx + kMbCap);
            __syncthreads();
#if !defined(SVO_K2V_KEEP_WAVES)
            if (retire && !preload_next && wave != 0) {  // (not in the debug kernel: kRetire false)
                retired = true;
                return;
            }
#endif
            did_preload = preload_next;
            if (preload_next && wave != 0) {
                load_raw(src);
                stage_wave0(src);
            }
            if (wave == 0) {
                uint32_t nw = 0;
                wave_rounds(seg, sh.mbx + kOneWave, nw);
                if (tid == 0) {
                    if (l - f <= 3) {  // std::__insertion_sort of the last <= 3
                        const uint32_t n = l - f;
                        double t[3] = {0.0, 0.0, 0.0};
                        for (uint32_t i = 0; i < n; ++i) t[i] = seg[f - f0 + i];
                        sort3(t, n);
                        hi = t[nth - f];
                        lo = rec ? lo_val : (nth >= f + 1 ? t[nth - 1 - f] : 0.0);
                    } else {  // depth limit
                        heap_select_at(seg + (f - f0), l - f, nth + 1 - f, nth - f);
                        hi = seg[nth - f0];
                        lo = rec ? lo_val : (nth >= f0 + 1 ? seg[nth - 1 - f0] : 0.0);
                        if (dg) dg->heap[P] = 1;
                    }
                    if (dg) dg->nwave[P] = nw;
                }
            }
        }
        __syncthreads();  // seg / mailbox / gseg are reused by the next pass
        // wave 0's staged rows (the next pass writes the mailbox only after its first barrier, which wave 0
        // reaches after these reads have completed)
        if (did_preload && wave == 0) unstage_wave0();
        VSTAMP(7);
#if defined(SVO_STAMPS) && defined(SVO_STAMPS_WAVES)
        if (kStampOn && dg && lane == 0) {
#pragma unroll
            for (int i = 0; i < 12; ++i) {
                dg->phw[wave][i] += phacc[i];
                if (tid == 0) dg->ph[i] += phacc[i];
                phacc[i] = 0;
            }
        }
#endif
        if (dg && tid == 0) {
            dg->nblock[P] = nblock;
            dg->cyc[P] = clock64() - t0;
        }
    }
};

// computeMedian / computeMAD (src/algorithm.cpp:834-865) with the reference's post-state; every thread
// returns med and mad.  M slots, n visible.
template <class L, bool kRetire>  // kRetire: waves 1-7 end after the last pass's dump (the product kernel only)
__device__ __forceinline__ void refv_robust_scale(const double* src, VShared<L>& sh, double* gseg, VDiag* dg, uint32_t M,
                                                  uint32_t n, double& med, double& mad) {
    L::Rows::fence();
    VSel<L> s{sh, gseg, (uint32_t)((M + 63u) / 64u * 64u), dg};
    s.M = M;
    s.nth = n / 2;
    s.tid = (int)threadIdx.x;
    s.lane = s.tid & 63;
    s.wave = (int)uni((uint32_t)(s.tid >> 6));
    const bool even = (M & 1u) == 0 && s.nth >= 1;  // mid == 0 (UB in the reference) reads vec[mid]
    double m0 = 0.0;
    bool pre = false;
    for (int P = 0; P < 2; ++P) {  // one copy of the selection for both passes
        s.P = P;
        double lo = 0.0, hi = 0.0;
        bool did = false, retired = false;
        s.select(src, P == 1, m0, pre, P == 0 && L::kPreload, hi, lo, did, kRetire && P == 1, retired);
        if (retired) return;  // (waves 1-7 after the last pass's dump: only thread 0's med / mad are used)
        pre = did;
        if (s.tid == 0) sh.bcd = even ? (lo + hi) / 2.0 : hi;
        __syncthreads();
        const double r = uni(sh.bcd);
        __syncthreads();
        if (P == 0) m0 = r;
        else mad = r;
    }
    med = m0;
}

template <class L>
__device__ __forceinline__ void scale_refv_pair(const AlignArgs& a, VShared<L>& sh) {
    const int pair = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    PairState& S = a.state[pair];
    if (!S.active) return;
    const PairDesc& P = a.pairs[pair];
    const int nf = P.n_ref + P.n_kf;
    const uint32_t M = (uint32_t)nf * (uint32_t)a.area;
    const uint8_t* __restrict__ fvis = a.fvis + (int64_t)pair * a.max_f;
    uint32_t nrv = 0, ncv = 0;
    for (int f = tid; f < nf; f += kVT) {
        const uint8_t v = fvis[f];
        nrv += v & 1;
        ncv += v >> 1;
    }
    nrv = wave_sum_u(nrv);
    ncv = wave_sum_u(ncv);
    if (lane == 0) { sh.tmp[wave] = nrv; sh.tmp[kVW + wave] = ncv; }
    __syncthreads();
    nrv = 0; ncv = 0;
    for (int w = 0; w < kVW; ++w) { nrv += sh.tmp[w]; ncv += sh.tmp[kVW + w]; }
    const uint32_t n = ncv * (uint32_t)a.area;
    double med = kDblMax, mad = 0.0;  // n == 0: every slot is DBL_MAX in the reference
    if (n > 0)
        refv_robust_scale<L, true>(a.scratch + (int64_t)pair * a.key_stride, sh,
                             reinterpret_cast<double*>(a.sel + (int64_t)pair * a.sel_stride), nullptr, M, n, med, mad);
    if (tid == 0) {
        double sigma = 1.482602218505602 * mad;
        if (sigma <= 2.220446049250313e-16) sigma = 2.220446049250313e-16;
        S.med = med;
        S.mad = mad;
        S.sigma = sigma;
        S.c = 4.6851 * sigma;
        S.n = n;
        S.n_ref_vis = nrv;
        S.scale_kernel = SVO_SCALE_K2V;
    }
}

}  // namespace

// K2V: one 512-thread workgroup per pair, one pair per CU (all of its registers and ~160 KB of LDS); one
// instantiation per register layout
template <class L>
__global__ void __launch_bounds__(kVT, 1) align_scale_refv_kernel(AlignArgs a, int level) {
    __shared__ VShared<L> sh;
    (void)level;
    SVO_TL_SCOPE(k2v, kTlK2V, level, a.pair_base);
    scale_refv_pair<L>(a, sh);
}
template __global__ void align_scale_refv_kernel<LayA>(AlignArgs, int);
template __global__ void align_scale_refv_kernel<LayB>(AlignArgs, int);
template __global__ void align_scale_refv_kernel<LayC>(AlignArgs, int);

// svo_debug_robust_scale: the same selection on an arbitrary vector (one workgroup); out[0..1] med / mad,
// out[2..] diagnostics (rounds, chunked rounds, heap selects, cycles per pass)
template <class L>
__global__ void __launch_bounds__(kVT, 1) debug_robust_scale_v_kernel(const double* v, uint32_t M, uint32_t n, double* gseg,
                                                                      double* out, double* trace, uint32_t trcap) {
    __shared__ VShared<L> sh;
    __shared__ VDiag dg;
    if (threadIdx.x == 0) {
        dg = VDiag{};
        dg.tr = trace;
        dg.trcap = trcap;
    }
    __syncthreads();
    double med = 0.0, mad = 0.0;
    refv_robust_scale<L, false>(v, sh, gseg, &dg, M, n, med, mad);
    if (threadIdx.x == 0) {
        out[0] = med;
        out[1] = mad;
        for (int P = 0; P < 2; ++P) {
            out[2 + 5 * P] = (double)dg.cyc[P];
            out[3 + 5 * P] = (double)dg.nblock[P];
            out[4 + 5 * P] = (double)dg.nwave[P];
            out[5 + 5 * P] = (double)dg.heap[P];
            out[6 + 5 * P] = (double)dg.nchunk[P];
        }
        for (int i = 0; i < 12; ++i) out[12 + i] = (double)dg.ph[i];
#if defined(SVO_STAMPS_WAVES)
        for (int i = 0; i < 128; ++i) out[24 + i] = i < 12 * kVW ? (double)dg.phw[i / 12][i % 12] : -1.0;
#else
        for (int i = 0; i < 128; ++i) out[24 + i] = i / 2 < (int)dg.nlog ? (double)dg.log[i / 2][i % 2] : -1.0;
#endif
    }
}

// svo_debug_robust_scale with out_len 2: the product kernel's code path (its layouts, 2048-position one-wave rounds,
// waves 1-7 retiring) on an arbitrary vector; out[0..1] med / mad
template <class L>
__global__ void __launch_bounds__(kVT, 1) plain_robust_scale_v_kernel(const double* v, uint32_t M, uint32_t n, double* gseg,
                                                                      double* out) {
    __shared__ VShared<L> sh;
    double med = 0.0, mad = 0.0;
    refv_robust_scale<L, true>(v, sh, gseg, nullptr, M, n, med, mad);
    if (threadIdx.x == 0) {
        out[0] = med;
        out[1] = mad;
    }
}

int64_t refv_max_slots() { return LayC::kCap; }
// the smaller layout (more mailbox, the MAD rows preloaded) whenever every pair of the launch fits it
void launch_scale_refv(const AlignArgs& a, int level, hipStream_t s) {
    if ((uint32_t)a.max_slots <= LayA::kCap)
        hipLaunchKernelGGL(align_scale_refv_kernel<LayA>, dim3(a.n_pairs), dim3(kVT), 0, s, a, level);
    else if ((uint32_t)a.max_slots <= LayB::kCap)
        hipLaunchKernelGGL(align_scale_refv_kernel<LayB>, dim3(a.n_pairs), dim3(kVT), 0, s, a, level);
    else
        hipLaunchKernelGGL(align_scale_refv_kernel<LayC>, dim3(a.n_pairs), dim3(kVT), 0, s, a, level);
}
void launch_debug_robust_scale_v(const double* v, uint32_t M, uint32_t n, double* gseg, double* out, double* trace,
                                 uint32_t trcap, hipStream_t s, bool plain) {
    if (plain) {
        if (M <= LayA::kCap)
            hipLaunchKernelGGL(plain_robust_scale_v_kernel<LayA>, dim3(1), dim3(kVT), 0, s, v, M, n, gseg, out);
        else if (M <= LayB::kCap)
            hipLaunchKernelGGL(plain_robust_scale_v_kernel<LayB>, dim3(1), dim3(kVT), 0, s, v, M, n, gseg, out);
        else
            hipLaunchKernelGGL(plain_robust_scale_v_kernel<LayC>, dim3(1), dim3(kVT), 0, s, v, M, n, gseg, out);
        return;
    }
    if (M <= LayADbg::kCap)
        hipLaunchKernelGGL(debug_robust_scale_v_kernel<LayADbg>, dim3(1), dim3(kVT), 0, s, v, M, n, gseg, out, trace, trcap);
    else if (M <= LayBDbg::kCap)
        hipLaunchKernelGGL(debug_robust_scale_v_kernel<LayBDbg>, dim3(1), dim3(kVT), 0, s, v, M, n, gseg, out, trace, trcap);
    else
        hipLaunchKernelGGL(debug_robust_scale_v_kernel<LayC>, dim3(1), dim3(kVT), 0, s, v, M, n, gseg, out, trace, trcap);
}

}  // namespace svo
