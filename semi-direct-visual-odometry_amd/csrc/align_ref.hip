// align_ref.hip — K2R: the reference's robust scale bit for bit (median_mode SVO_MEDIAN_REFERENCE).
//
// Optimizer::tukeyWeighting (src/optimizer.cpp:485-514) takes sigma = 1.482602218505602 * MAD with
// algorithm::computeMedian (src/algorithm.cpp:834-853) on the FULL residual vector (n_features * patch^2
// slots in feature-major order, invisible slots = DBL_MAX): std::nth_element(vec, vec + n/2), then, for an
// even total length, (vec[n/2 - 1] + vec[n/2]) / 2 — where vec[n/2 - 1] is whatever libstdc++'s
// introselect left there, not always the (n/2 - 1)-th order statistic.  The MAD is the
// same call on |r_i - median| in the original order (:855-865).
//
// K2R re-runs libstdc++'s introselect (stl_algo.h __introselect, GCC 11) on the device, one 512-thread
// workgroup per pair, two pairs per CU.  Elements are the exact residuals (doubles, written by K1 in the
// reference's slot order), so every comparison is the reference's own `<`.  Each partition round is the
// parallel form tests/cpp/introselect_model.cpp derives and checks against std::nth_element:
//   median of three (first+1, first+S/2, last-1) moved to first, pivot p;
//   GE = positions in [first+1, last) with !(a < p), LE = positions in [first, last) with !(p < a);
//   the Hoare loop swaps the k-th GE from the left (L_k) with the k-th LE from the right (R_k) for k <= Ks,
//   Ks = max over split points t of min(#GE before t, #LE from t on), and returns
//   cut = min(L_{Ks+1}, R_{Ks}).
// Only the side introselect continues with is materialised: its swap targets take their partners' values
// through a mailbox indexed by k.
//
// Layout.  Positions are grouped in steps of 64 (one wave instruction) and blocks of 8 steps; block b is
// owned by wave b % 8 in every round, so a wave only ever reads and writes the positions it owns and a
// round needs three barriers: after the classification sweep (per-step GE / LE ballots and counts, per-block
// totals), after the mailbox writes, after the target writes (which also publish the next round's pivot
// candidates).  Between the first two, every wave scans the block totals redundantly and finds the crossing,
// Ks, L_{Ks+1} and R_{Ks} by block -> step -> bit searches (two dependent record reads each).  Segments of
// <= 11 blocks live in LDS (values, mailbox, step records); larger ones in the pair's global scratch, the
// first round straight from K1's residuals.  Segments of <= 64 elements run on one wave from registers;
// the depth limit falls back to the restated heap select (one lane; adversarial inputs only), the last
// <= 3 values are sorted.  vec[n/2 - 1] is recorded at the round whose cut lands exactly on n/2 (that slot is
// never touched again), or read after the final sort.
#include <cstdlib>

#include "svo_internal.h"
#include "svo_math.h"
#include "svo_wave.h"
#include "ref_common.h"

namespace svo {

namespace {

using namespace refsel;

constexpr uint32_t kBlk = 512;               // positions per block (8 steps of 64), owned by wave block % TW
// TW waves per pair: 8 (512 threads, two pairs per CU: batches of more than 128 pairs per launch) or 16
// (1024 threads, one pair per CU with a 20-block LDS segment: small batches, the per-frame latency)
template <int TW>
struct Geo {
    static constexpr int RT = 64 * TW;
    static constexpr uint32_t Cap = (TW == 8 ? 9u : 20u) * kBlk;  // LDS segment capacity (block-aligned base)
};
constexpr uint32_t kRecSteps = 1024;         // LDS step records (absolute steps): vectors of <= 64512 slots
constexpr int kLogCap = 60;                  // diagnostics: block rounds logged per call


template <int NB, int TW>
struct RefShared {
    static constexpr uint32_t kRec = NB <= 2 ? kRecSteps : 1;  // (NB > 2: the records are global)
    static constexpr uint32_t kCap = Geo<TW>::Cap;
    double seg[kCap];               // the segment, from position `base`
    double mb[kCap / 2];            // mailbox of LDS rounds (Ks <= S / 2) and of the one-wave rounds
    uint64_t msk[kRec][2];          // per step: GE, LE ballots
    uint32_t cnt[kRec];             // per step: #GE | #LE << 16
    uint32_t btot[64 * NB];         // per block: #GE | #LE << 16
    double cand[4];                 // the next round's A, B, C, first values (published by their owners)
    double bcd;                     // broadcast (median between the passes)
    uint32_t bcu[6];                // broadcast of the one-wave rounds' state
    double bclo;
};

struct Diag {  // svo_debug_robust_scale diagnostics (compiled out of the product)
    uint64_t cyc[2];
    uint32_t nblock[2], nlane[2], heap[2];
    uint32_t log[kLogCap][3];  // block rounds: S, where, cycles
    uint32_t nlog;
    uint64_t ph[2][8];  // cycles per phase of the block rounds (thread 0), [global, LDS]
};

__device__ __forceinline__ double bperm(double v, uint32_t src_lane) {
    const uint2 u = __builtin_bit_cast(uint2, v);
    const int a = (int)(src_lane * 4u);
    return __builtin_bit_cast(double, make_uint2((uint32_t)__builtin_amdgcn_ds_bpermute(a, (int)u.x),
                                                 (uint32_t)__builtin_amdgcn_ds_bpermute(a, (int)u.y)));
}

// NB: rows of 64 blocks held in registers by the block scans (2: M <= 64512, 17: M <= 524288).  With NB = 2
// the step records live in LDS (absolute steps), else in the pair's global scratch.
template <int NB, int TW, bool kSt>
struct RefSel {
    static constexpr bool kRecLds = NB <= 2;
    static constexpr int kRW = TW, kRT = Geo<TW>::RT;
    static constexpr uint32_t kCap = Geo<TW>::Cap;
    using Sh = RefShared<NB, TW>;
    Sh& sh;
    Diag* dg;
    const double* src;  // the pass's source vector (K1's residuals, reference slot order), read-only
    double* gseg;       // pair's global segment (absolute positions)
    double* gmb;        // global mailbox
    uint64_t* gmsk;     // global step records (NB > 2)
    uint32_t* gcnt;
    uint32_t M, nth;
    int tid, lane, wave;
    int P;              // pass: 0 median, 1 MAD (values |r - med|)
    double med;
    // block-uniform selection state
    uint32_t f, l, base;
    int where, depth;
    bool rec;
    double lo_val;
    double p, x0;       // the round's pivot (at f after the median-of-three swap) and the value moved to ch
    uint32_t ch;
    const double* sp;   // storage: value(q) = sp[q - sb] (a flat pointer: LDS or global)
    uint32_t sb;
    bool xf;            // reading K1's array in pass 1: |r - med| on load
    // block scan of the current round (lane j of row r: block b0 + 64 r + j)
    uint32_t bpg[NB], bpl[NB], btg[NB], btl[NB];
    uint32_t totG, totL;

    // ---------------------------------------------------------------- storage and records
    __device__ __forceinline__ void set_storage(int w, uint32_t b) {
        where = w;
        base = b;
        sp = w == kLds ? sh.seg : (w == kGlb ? gseg : src);
        sb = w == kLds ? b : 0u;
        xf = w == kSrc && P == 1;
    }
    __device__ __forceinline__ double ld(uint32_t q) const {
        const double v = sp[q - sb];
        return xf ? fabs(v - med) : v;  // src/algorithm.cpp:860-863 (DBL_MAX stays DBL_MAX)
    }
    // the value at q after the round's median-of-three swap
    __device__ __forceinline__ double vpre(uint32_t q) const { return q == f ? p : (q == ch ? x0 : ld(q)); }
    __device__ __forceinline__ uint64_t* mrec(uint32_t s) const {
        if constexpr (kRecLds) return &sh.msk[s][0];
        else return gmsk + 2 * (size_t)s;
    }
    __device__ __forceinline__ uint32_t* crec(uint32_t s) const {
        if constexpr (kRecLds) return &sh.cnt[s];
        else return gcnt + s;
    }
    __device__ __forceinline__ void choose(double a, double b, double c, double x) {
        const uint32_t S = l - f;
        median3(a, b, c, f + 1, f + S / 2, l - 1, ch, p);
        x0 = x;
        p = uni(p); x0 = uni(x0); ch = uni(ch);
    }
    __device__ __forceinline__ void pivot_from_storage() {
        const uint32_t S = l - f;
        choose(uni(ld(f + 1)), uni(ld(f + S / 2)), uni(ld(l - 1)), uni(ld(f)));
    }
    // element i of a row array at a uniform block index
    __device__ __forceinline__ uint32_t rrd(const uint32_t (&a)[NB], uint32_t i) const {
        uint32_t v = 0;
#pragma unroll
        for (int r = 0; r < NB; ++r)
            if ((i >> 6) == (uint32_t)r) v = lane_read(a[r], (int)(i & 63u));
        return v;
    }
    __device__ __forceinline__ uint32_t first_own(uint32_t b0) const {
        return b0 + (uint32_t)(((int)wave - (int)(b0 % kRW) + kRW) % kRW);
    }
    // a block's 8 step records (lane j < 8: step 8 b + j) and their exclusive GE / LE prefixes in the block
    __device__ __forceinline__ void block_recs(uint32_t b, uint64_t& mg, uint64_t& ml, uint32_t& eg, uint32_t& el) const {
        uint32_t c8 = 0;
        mg = ml = 0;
        if (lane < 8) {
            const uint64_t* mr = mrec(8 * b + (uint32_t)lane);
            mg = mr[0];
            ml = mr[1];
            c8 = *crec(8 * b + (uint32_t)lane);
        }
        const uint32_t sg = c8 & 0xFFFFu, sl = c8 >> 16;
        eg = wave_incl_scan(sg) - sg;
        el = wave_incl_scan(sl) - sl;
    }

    // ---------------------------------------------------------------- classification sweep (own blocks)
    // Loads are branch-free (lanes outside the segment read position f): a load under an exec branch with
    // its use inside the branch waits for it before the next one is issued
    __device__ __forceinline__ double xform(double t) const { return xf ? fabs(t - med) : t; }
    __device__ __forceinline__ void load8(uint32_t b, double (&v)[8]) const {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const uint32_t q = b * kBlk + 64u * (uint32_t)j + (uint32_t)lane;
            v[j] = sp[((q >= f && q < l) ? q : f) - sb];  // raw: fix() at the use, after the next loads
        }
    }
    // a raw load at q as the round sees it: the pass-1 transform and the median-of-three swap
    __device__ __forceinline__ double fix(uint32_t q, double t) const { return q == f ? p : (q == ch ? x0 : xform(t)); }
    __device__ __forceinline__ void classify8(uint32_t b, const double (&raw)[8]) {
        uint32_t mgl = 0, mgh = 0, mll = 0, mlh = 0, cv = 0, tg = 0, tl = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const uint32_t q = b * kBlk + 64u * (uint32_t)j + (uint32_t)lane;
            const bool in = q >= f && q < l;
            const double v = fix(q, raw[j]);
            const uint64_t ge = __ballot(in && q != f && !(v < p));
            const uint64_t le = __ballot(in && !(p < v));
            const uint32_t cg = popc(ge), cl = popc(le);
            mgl = lane_write(mgl, (uint32_t)ge, (uint32_t)j);
            mgh = lane_write(mgh, (uint32_t)(ge >> 32), (uint32_t)j);
            mll = lane_write(mll, (uint32_t)le, (uint32_t)j);
            mlh = lane_write(mlh, (uint32_t)(le >> 32), (uint32_t)j);
            cv = lane_write(cv, cg | (cl << 16), (uint32_t)j);
            tg += cg;
            tl += cl;
        }
        if (lane < 8) {
            uint64_t* mr = mrec(8 * b + (uint32_t)lane);
            mr[0] = ((uint64_t)mgh << 32) | mgl;
            mr[1] = ((uint64_t)mlh << 32) | mll;
            *crec(8 * b + (uint32_t)lane) = cv;
        }
        if (lane == 0) sh.btot[b] = tg | (tl << 16);
    }
    // two blocks per pass: their 16 loads per lane are in flight together, then both are classified
    __device__ __forceinline__ void sweep(uint32_t b0, uint32_t b1) {
        for (uint32_t b = first_own(b0); b <= b1; b += 2 * kRW) {
            double v[2][8];
            const bool two = b + kRW <= b1;
            load8(b, v[0]);
            if (two) load8(b + kRW, v[1]);
            classify8(b, v[0]);
            if (two) classify8(b + kRW, v[1]);
        }
    }

    // ---------------------------------------------------------------- exchange stages (two blocks per pass)
    // sources: the mailbox slot of each source lane and its raw value
    __device__ __forceinline__ void src_stage(uint32_t b, uint32_t b0, uint32_t ks, bool right, uint32_t (&ns)[8],
                                              double (&nv)[8]) const {
        const uint32_t me = (uint32_t)lane, rb = b - b0;
        const uint32_t gpb = rrd(bpg, rb), lpb = rrd(bpl, rb), ltb = rrd(btl, rb);
        const bool any = right ? gpb < ks : lpb + ltb + ks >= totL + 1u;
#pragma unroll
        for (int j = 0; j < 8; ++j) ns[j] = kNone;
        if (!any) return;
        uint64_t mg, ml;
        uint32_t eg, el;
        block_recs(b, mg, ml, eg, el);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const uint64_t ge = lane_read64(mg, j), le = lane_read64(ml, j);
            const uint32_t q = b * kBlk + 64u * (uint32_t)j + me;
            if (right) {
                const uint32_t k = gpb + lane_read(eg, j) + lanes_below(ge) + 1u;
                if (((ge >> me) & 1ull) && k <= ks) ns[j] = k - 1u;
            } else {
                const uint32_t k = totL - (lpb + lane_read(el, j) + lanes_below(le));
                if (((le >> me) & 1ull) && k <= ks) ns[j] = k - 1u;
            }
            nv[j] = sp[(ns[j] != kNone ? q : f) - sb];  // raw (fixed at the store)
        }
    }
    __device__ __forceinline__ void src_store(uint32_t b, double* mbp, const uint32_t (&ns)[8], const double (&nv)[8]) const {
#pragma unroll
        for (int j = 0; j < 8; ++j)
            if (ns[j] != kNone) mbp[ns[j]] = fix(b * kBlk + 64u * (uint32_t)j + (uint32_t)lane, nv[j]);
    }
    // targets: one load per lane (the mailbox for a target, the storage where the value must be written or
    // published, a common dummy otherwise); flags bit 0 write, bit 1 publish, bit 2 the value is the mailbox's
    struct Tgt {
        uint32_t nf, nl, cA, cB, cC, cF, ks;
        bool right, copy;
        const double* mbp;
    };
    __device__ __forceinline__ void tgt_stage(uint32_t b, uint32_t b0, const Tgt& t, uint32_t (&fl)[8], double (&nv)[8]) const {
        const uint32_t me = (uint32_t)lane, rb = b - b0;
        const uint32_t gpb = rrd(bpg, rb), lpb = rrd(bpl, rb);
        uint64_t mg, ml;
        uint32_t eg, el;
        block_recs(b, mg, ml, eg, el);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const uint64_t ge = lane_read64(mg, j), le = lane_read64(ml, j);
            const uint32_t q = b * kBlk + 64u * (uint32_t)j + me;
            const bool in = q >= t.nf && q < t.nl;
            uint32_t k = kNone;
            if (t.right) {
                const uint32_t kk = totL - (lpb + lane_read(el, j) + lanes_below(le));
                if (((le >> me) & 1ull) && kk <= t.ks) k = kk;
            } else {
                const uint32_t kk = gpb + lane_read(eg, j) + lanes_below(ge) + 1u;
                if (((ge >> me) & 1ull) && kk <= t.ks) k = kk;
            }
            const bool tg = in && k != kNone;
            const bool pub = in && (q == t.cA || q == t.cB || q == t.cC || q == t.cF);
            const bool wr = in && (tg || t.copy || q == f || q == ch);
            fl[j] = (wr ? 1u : 0u) | (pub ? 2u : 0u) | (tg ? 4u : 0u);
            const double* a = tg ? t.mbp + (k - 1) : sp + (((wr || pub) ? q : t.nf) - sb);
            nv[j] = *a;
        }
    }
    __device__ __forceinline__ void tgt_store(uint32_t b, const Tgt& t, double* dp, uint32_t db, const uint32_t (&fl)[8],
                                              const double (&nv)[8]) const {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const uint32_t q = b * kBlk + 64u * (uint32_t)j + (uint32_t)lane;
            const double x = (fl[j] & 4u) ? nv[j] : fix(q, nv[j]);
            if (fl[j] & 1u) dp[q - db] = x;
            if (fl[j] & 2u) sh.cand[q == t.cA ? 0 : q == t.cB ? 1 : q == t.cC ? 2 : 3] = x;
        }
    }

    // ---------------------------------------------------------------- block scan, crossing, rank searches
    __device__ __forceinline__ void block_scan(uint32_t b0, uint32_t nblk) {
        uint32_t cg = 0, cl = 0;
#pragma unroll
        for (int r = 0; r < NB; ++r) {
            bpg[r] = bpl[r] = btg[r] = btl[r] = 0;
            if (64u * (uint32_t)r < nblk) {
                const uint32_t rb = 64u * (uint32_t)r + (uint32_t)lane;
                const uint32_t t = rb < nblk ? sh.btot[b0 + rb] : 0u;
                const uint32_t tg = t & 0xFFFFu, tl = t >> 16;
                const uint32_t ig = wave_incl_scan(tg), il = wave_incl_scan(tl);
                bpg[r] = cg + ig - tg;
                bpl[r] = cl + il - tl;
                btg[r] = tg;
                btl[r] = tl;
                cg += lane_read(ig, 63);
                cl += lane_read(il, 63);
            }
        }
        totG = uni(cg);
        totL = uni(cl);
    }
    // Ks = max(G(t* - 1), Lc(t*)), t* the first split point with G(t) >= Lc(t)
    __device__ __forceinline__ uint32_t crossing(uint32_t b0, uint32_t nblk) const {
        uint32_t tb = nblk - 1;
        bool found = false;
#pragma unroll
        for (int r = 0; r < NB; ++r) {
            if (!found && 64u * (uint32_t)r < nblk) {
                const uint32_t rb = 64u * (uint32_t)r + (uint32_t)lane;
                const uint64_t m = __ballot(rb >= 1 && rb < nblk && bpg[r] >= totL - bpl[r]);
                if (m) {
                    tb = 64u * (uint32_t)r + (uint32_t)__builtin_ctzll(m) - 1u;
                    found = true;
                }
            }
        }
        tb = uni(tb);
        uint32_t gcar = rrd(bpg, tb), lcar = totL - rrd(bpl, tb);
        uint64_t mg, ml;
        uint32_t eg, el;
        block_recs(b0 + tb, mg, ml, eg, el);
        const uint64_t m = __ballot(lane >= 1 && lane < 8 && gcar + eg >= lcar - el);
        const uint32_t ts = m ? (uint32_t)__builtin_ctzll(m) - 1u : 7u;
        gcar += lane_read(eg, (int)ts);
        lcar -= lane_read(el, (int)ts);
        const uint64_t a = lane_read64(mg, (int)ts), bb = lane_read64(ml, (int)ts);
        uint32_t lo = 1, hi = 64;  // smallest bit split b with G(b) >= Lc(b) inside the step
        while (lo < hi) {
            const uint32_t mid = (lo + hi) / 2;
            const uint64_t lm = low_mask(mid);
            if (gcar + popc(a & lm) >= lcar - popc(bb & lm)) hi = mid;
            else lo = mid + 1;
        }
        const uint32_t g1 = gcar + popc(a & low_mask(lo - 1));
        const uint32_t l2 = lcar - popc(bb & low_mask(lo));
        return g1 > l2 ? g1 : l2;
    }
    // the rank-th (1-based) GE (kind 0) or LE (kind 1) position from the left, kNone if there is none
    __device__ __forceinline__ uint32_t pos_of(int kind, uint32_t rank, uint32_t b0, uint32_t nblk) const {
        if (rank == 0 || rank > (kind ? totL : totG)) return kNone;
        uint32_t rb = kNone;
#pragma unroll
        for (int r = 0; r < NB; ++r) {
            if (rb == kNone && 64u * (uint32_t)r < nblk) {
                const uint32_t inc = kind ? bpl[r] + btl[r] : bpg[r] + btg[r];
                const uint64_t m = __ballot(64u * (uint32_t)r + (uint32_t)lane < nblk && inc >= rank);
                if (m) rb = 64u * (uint32_t)r + (uint32_t)__builtin_ctzll(m);
            }
        }
        rb = uni(rb);
        uint32_t pre = kind ? rrd(bpl, rb) : rrd(bpg, rb);
        uint64_t mg, ml;
        uint32_t eg, el;
        block_recs(b0 + rb, mg, ml, eg, el);
        const uint32_t ex = kind ? el : eg;
        const uint64_t m = __ballot(lane < 8 && pre + ex < rank);  // steps starting below the rank
        const uint32_t j = 63u - (uint32_t)__builtin_clzll(m);    // the last of them holds it
        pre += lane_read(ex, (int)j);
        const uint64_t mk = kind ? lane_read64(ml, (int)j) : lane_read64(mg, (int)j);
        return (8 * (b0 + rb) + j) * 64u + select_bit(mk, rank - pre - 1u);
    }

    // ---------------------------------------------------------------- one partition round (8 waves)
    __device__ __forceinline__ void round() {
        const uint32_t b0 = f / kBlk, b1 = (l - 1) / kBlk, nblk = b1 - b0 + 1;
        uint64_t tp = kSt ? clock64() : 0;
        const int pw = where == kLds ? 1 : 0;
        auto phase = [&](int i) {
            if (kSt && tid == 0) { const uint64_t t = clock64(); dg->ph[pw][i] += t - tp; tp = t; }
        };
        sweep(b0, b1);
        phase(0);
        if (!kRecLds) __threadfence_block();
        __syncthreads();
        phase(1);
        block_scan(b0, nblk);
        const uint32_t ks = uni(crossing(b0, nblk));
        const uint32_t lk1 = uni(pos_of(0, ks + 1, b0, nblk));
        const uint32_t rk = ks >= 1 ? uni(pos_of(1, totL - ks + 1, b0, nblk)) : kNone;
        const uint32_t cut = lk1 < rk ? lk1 : rk;
        const bool right = cut <= nth;  // the side introselect continues with
        const uint32_t nf = right ? cut : f, nl = right ? l : cut;
        if (cut == nth && !rec) {  // vec[nth - 1] after this round: only L_{Ks} can be cut - 1
            const uint32_t lk = ks >= 1 ? uni(pos_of(0, ks, b0, nblk)) : kNone;
            lo_val = uni(lk == cut - 1 ? vpre(rk) : vpre(cut - 1));
            rec = true;
        }
        phase(2);
        int dst = where == kSrc ? kGlb : where;
        uint32_t nbase = base;
        if (where != kLds && nl - (nf & ~(kBlk - 1)) <= kCap) {
            dst = kLds;
            nbase = nf & ~(kBlk - 1);
        }
        const bool copy = dst != where;
        // the LDS mailbox whenever the round's Ks swaps fit it (global rounds included: their values still
        // come from and go to global storage, but the exchange skips a global store / load pair)
        double* const mbp = (where == kLds || ks <= kCap / 2) ? sh.mb : gmb;
        // ---- sources to the mailbox: right side kept -> L_k's value at k - 1; left side kept -> R_k's.
        // Two blocks per pass: their loads are in flight together, then stored.
        for (uint32_t b = first_own(b0); b <= b1; b += 2 * kRW) {
            uint32_t ns[2][8];
            double nv[2][8];
            const bool two = b + kRW <= b1;
            src_stage(b, b0, ks, right, ns[0], nv[0]);
            if (two) src_stage(b + kRW, b0, ks, right, ns[1], nv[1]);
            src_store(b, mbp, ns[0], nv[0]);
            if (two) src_store(b + kRW, mbp, ns[1], nv[1]);
        }
        phase(3);
        if (where != kLds) __threadfence_block();
        __syncthreads();
        phase(4);
        // ---- the kept side: targets take the mailbox, the rest stays (or moves to the new storage); the
        // owners of the next round's A, B, C and first publish their values.  Pipelined like the sources.
        const uint32_t nS = nl - nf;
        const uint32_t cA = nS >= 4 ? nf + 1 : kNone, cB = nS >= 4 ? nf + nS / 2 : kNone, cC = nS >= 4 ? nl - 1 : kNone,
                       cF = nS >= 4 ? nf : kNone;
        double* const dp = dst == kLds ? sh.seg : gseg;
        const uint32_t db = dst == kLds ? nbase : 0u;
        {
            Tgt t;
            t.nf = nf; t.nl = nl; t.cA = cA; t.cB = cB; t.cC = cC; t.cF = cF; t.ks = ks;
            t.right = right; t.copy = copy; t.mbp = mbp;
            const uint32_t nb0 = nf / kBlk, nb1 = (nl - 1) / kBlk;
            for (uint32_t b = first_own(nb0); b <= nb1; b += 2 * kRW) {
                uint32_t fl[2][8];
                double nv[2][8];
                const bool two = b + kRW <= nb1;
                tgt_stage(b, b0, t, fl[0], nv[0]);
                if (two) tgt_stage(b + kRW, b0, t, fl[1], nv[1]);
                tgt_store(b, t, dp, db, fl[0], nv[0]);
                if (two) tgt_store(b + kRW, t, dp, db, fl[1], nv[1]);
            }
        }
        phase(5);
        if (dst != kLds) __threadfence_block();
        __syncthreads();
        phase(6);
        f = nf;
        l = nl;
        set_storage(dst, nbase);
        if (nS >= 4) choose(uni(sh.cand[0]), uni(sh.cand[1]), uni(sh.cand[2]), uni(sh.cand[3]));
        phase(7);
    }

    // ---------------------------------------------------------------- rounds of a segment of <= 512 elements
    // One wave, no barriers: lane l of register j holds position f0 + 64 j + l; the median of three by
    // readlane, the masks by compares, the counts / crossing / rank searches on scalars, the swaps through a
    // wave-private LDS mailbox (a wave's LDS accesses complete in program order); vec[nth - 1] recorded from
    // registers; written back once at the end.  Stops at <= 3 elements or depth 0.
    static __device__ __forceinline__ double vat(const double (&v)[8], uint32_t i) {
        double r = 0.0;
#pragma unroll
        for (int j = 0; j < 8; ++j)
            if ((i >> 6) == (uint32_t)j) r = lane_read(v[j], (int)(i & 63u));
        return r;
    }
    __device__ __forceinline__ void vset(double (&v)[8], uint32_t i, double x) const {
#pragma unroll
        for (int j = 0; j < 8; ++j)
            if ((i >> 6) == (uint32_t)j && (uint32_t)lane == (i & 63u)) v[j] = x;
    }
    __device__ __forceinline__ void wave_rounds(uint32_t& nrounds) {
        const uint32_t f0 = f, S0 = l - f, me = (uint32_t)lane;
        double v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const uint32_t i = 64u * (uint32_t)j + me;
            v[j] = sp[f0 + (i < S0 ? i : 0u) - sb];
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = 64u * (uint32_t)j + me < S0 ? xform(v[j]) : kDblMax;
        uint32_t fr = 0, lr = S0;
        const uint32_t nrel = nth - f0;
        double* const mb = sh.mb;
        while (lr - fr > 3 && depth > 0) {
            --depth;
            ++nrounds;
            const uint32_t A = fr + 1, B = fr + (lr - fr) / 2, C = lr - 1;
            const double a = vat(v, A), b = vat(v, B), c = vat(v, C), xv = vat(v, fr);
            uint32_t chh;
            double pe;
            median3(a, b, c, A, B, C, chh, pe);
            pe = uni(pe);
            chh = uni(chh);
            vset(v, fr, pe);
            vset(v, chh, xv);
            uint64_t ge[8], le[8];
            uint32_t gp[8], lp[8];  // #GE / #LE before each step
            uint32_t tG = 0, tL = 0;
            // only the steps the segment touches do vector work (the later rounds span one or two)
            const uint32_t js = fr / 64u, je = (lr + 63u) / 64u;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const uint32_t i = 64u * (uint32_t)j + me;
                const bool in = i >= fr && i < lr;
                ge[j] = __ballot(in && i != fr && !(v[j] < pe));
                le[j] = __ballot(in && !(pe < v[j]));
                gp[j] = tG;
                lp[j] = tL;
                tG += popc(ge[j]);
                tL += popc(le[j]);
            }
            // crossing: the last step whose start has G < Lc (step 0: G = 0 < Lc), then its bit
            uint32_t gcar = 0, lcar = tL;
            uint64_t a0 = ge[0], b0m = le[0];
#pragma unroll
            for (int j = 1; j < 8; ++j)
                if (gp[j] < tL - lp[j]) { gcar = gp[j]; lcar = tL - lp[j]; a0 = ge[j]; b0m = le[j]; }
            uint32_t lo = 1, hi = 64;
            while (lo < hi) {
                const uint32_t mid = (lo + hi) / 2;
                const uint64_t lm = low_mask(mid);
                if (gcar + popc(a0 & lm) >= lcar - popc(b0m & lm)) hi = mid;
                else lo = mid + 1;
            }
            const uint32_t g1 = gcar + popc(a0 & low_mask(lo - 1)), l2 = lcar - popc(b0m & low_mask(lo));
            const uint32_t ks = g1 > l2 ? g1 : l2;
            auto rank_pos = [&](int kind, uint32_t rank) -> uint32_t {  // the last step starting below the rank
                if (rank == 0 || rank > (kind ? tL : tG)) return kNone;
                uint32_t pre = 0, jj = 0;
                uint64_t mk = kind ? le[0] : ge[0];
#pragma unroll
                for (int j = 1; j < 8; ++j) {
                    const uint32_t pj = kind ? lp[j] : gp[j];
                    if (pj < rank) { pre = pj; jj = (uint32_t)j; mk = kind ? le[j] : ge[j]; }
                }
                return 64u * jj + select_bit(mk, rank - pre - 1u);
            };
            const uint32_t lk1 = rank_pos(0, ks + 1), rk = ks >= 1 ? rank_pos(1, tL - ks + 1) : kNone;
            const uint32_t cut = lk1 < rk ? lk1 : rk;
            const bool right = cut <= nrel;
            if (cut == nrel && !rec && nrel >= 1) {
                const uint32_t lk = ks >= 1 ? rank_pos(0, ks) : kNone;
                lo_val = uni(vat(v, lk == cut - 1 ? rk : cut - 1));
                rec = true;
            }
            // sources to the mailbox, then the kept side's targets read it
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                if ((uint32_t)j < js || (uint32_t)j >= je) continue;
                uint32_t k = kNone;
                if (right) {
                    const uint32_t kk = gp[j] + lanes_below(ge[j]) + 1u;
                    if (((ge[j] >> me) & 1ull) && kk <= ks) k = kk;
                } else {
                    const uint32_t kk = tL - (lp[j] + lanes_below(le[j]));
                    if (((le[j] >> me) & 1ull) && kk <= ks) k = kk;
                }
                mb[k != kNone ? k - 1 : kCap / 2 - 64 + me] = v[j];  // (non-sources: a dummy slot per lane)
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                if ((uint32_t)j < js || (uint32_t)j >= je) continue;
                uint32_t k = kNone;
                if (right) {
                    const uint32_t kk = tL - (lp[j] + lanes_below(le[j]));
                    if (((le[j] >> me) & 1ull) && kk <= ks) k = kk;
                } else {
                    const uint32_t kk = gp[j] + lanes_below(ge[j]) + 1u;
                    if (((ge[j] >> me) & 1ull) && kk <= ks) k = kk;
                }
                const double x = mb[k != kNone ? k - 1 : kCap / 2 - 64 + me];
                v[j] = k != kNone ? x : v[j];
            }
            if (right) fr = cut;
            else lr = cut;
        }
        if (where == kSrc) set_storage(kLds, 0);  // a vector of <= 512 slots never left K1's array
        double* const dp = where == kLds ? sh.seg : gseg;
        const uint32_t db = where == kLds ? base : 0u;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const uint32_t i = 64u * (uint32_t)j + me;
            if (i < S0) dp[f0 + i - db] = v[j];
        }
        f = f0 + fr;
        l = f0 + lr;
    }

    // ---------------------------------------------------------------- std::nth_element(vec, vec + nth)
    // (vec[nth - 1], vec[nth]) of the post-state, on thread 0
    __device__ __forceinline__ void select(double& lo, double& hi) {
        f = 0; l = M; rec = false; lo_val = 0.0;
        set_storage(kSrc, 0);
        depth = M > 1 ? 2 * lg2(M) : 0;
        bool have = false;  // the pivot of [f, l) is known (published by the previous block round)
        uint32_t nblock = 0, heap = 0;
        const uint64_t t0 = kSt ? clock64() : 0;
        while (l - f > 3) {
            if (depth == 0) {
                if (tid == 0) heap_select_fn(sh.seg, base, gseg, where, f, l - f, nth + 1 - f, nth - f);
                heap = 1;
                __threadfence_block();
                __syncthreads();
                break;
            }
            if (l - f <= kBlk) {  // the rest on wave 0, from registers
                if (wave == 0) {
                    uint32_t nr = 0;
                    wave_rounds(nr);
                    if (lane == 0) {
                        sh.bcu[0] = f; sh.bcu[1] = l; sh.bcu[2] = (uint32_t)depth; sh.bcu[3] = rec ? 1u : 0u;
                        sh.bcu[4] = (uint32_t)where; sh.bcu[5] = base; sh.bclo = lo_val;
                        if (kSt) dg->nlane[P] += nr;
                    }
                }
                __threadfence_block();
                __syncthreads();
                f = uni(sh.bcu[0]); l = uni(sh.bcu[1]); depth = (int)uni(sh.bcu[2]); rec = uni(sh.bcu[3]) != 0;
                set_storage((int)uni(sh.bcu[4]), uni(sh.bcu[5]));
                lo_val = uni(sh.bclo);
                __syncthreads();
                have = false;
                continue;
            }
            if (!have) pivot_from_storage();
            --depth;
            const uint64_t tb = kSt ? clock64() : 0;
            const uint32_t S = l - f, w = (uint32_t)where;
            round();
            have = true;
            ++nblock;
            if (kSt && tid == 0 && dg->nlog < kLogCap) {
                dg->log[dg->nlog][0] = S; dg->log[dg->nlog][1] = w; dg->log[dg->nlog][2] = (uint32_t)(clock64() - tb);
                dg->nlog++;
            }
        }
        if (kSt && tid == 0) {
            dg->cyc[P] = clock64() - t0;
            dg->nblock[P] = nblock;
            dg->heap[P] = heap;
        }
        if (tid == 0) {
            if (l - f <= 3) {  // std::__insertion_sort of the last <= 3
                const uint32_t n = l - f;
                double v[3];
                for (uint32_t i = 0; i < n; ++i) v[i] = ld(f + i);
                for (uint32_t i = 1; i < n; ++i) {
                    const double x = v[i];
                    uint32_t j = i;
                    while (j > 0 && x < v[j - 1]) { v[j] = v[j - 1]; --j; }
                    v[j] = x;
                }
                hi = v[nth - f];
                if (nth >= 1) lo = rec ? lo_val : v[nth - 1 - f];
            } else {  // heap select ran
                hi = ld(nth);
                if (nth >= 1) lo = rec ? lo_val : ld(nth - 1);
            }
        }
    }
};

// computeMedian / computeMAD (src/algorithm.cpp:834-865) with the reference's post-state: thread 0 of the
// block gets med and mad.  M slots, n visible; sel: the pair's scratch (sel_stride u32).
template <int NB, int TW, bool kSt>
__device__ __forceinline__ void ref_robust_scale(const double* src, RefShared<NB, TW>& sh, Diag* dg, uint32_t* sel,
                                                 int64_t sel_stride, uint32_t M, uint32_t n, double& med, double& mad) {
    const int tid = (int)threadIdx.x;
    const int64_t mp = sel_stride / 4;  // positions the scratch holds (a multiple of kBlk, >= M + kBlk)
    RefSel<NB, TW, kSt> s{sh, dg};
    s.src = src;
    s.gseg = reinterpret_cast<double*>(sel);
    s.gmb = s.gseg + mp;
    s.gmsk = reinterpret_cast<uint64_t*>(s.gmb + mp / 2);
    s.gcnt = reinterpret_cast<uint32_t*>(s.gmsk + 2 * (mp / 64));
    s.M = M;
    s.nth = n / 2;
    s.tid = tid; s.lane = tid & 63; s.wave = (int)uni((uint32_t)(tid >> 6));
    s.med = 0.0;
    const bool even = (M & 1u) == 0 && s.nth >= 1;  // mid == 0 (UB in the reference) reads vec[mid]
    for (int P = 0; P < 2; ++P) {  // one copy of the selection for both passes
        s.P = P;
        double lo = 0.0, hi = 0.0;
        s.select(lo, hi);
        if (tid == 0) {
            const double v = even ? (lo + hi) / 2.0 : hi;
            if (P == 0) { sh.bcd = v; med = v; }
            else mad = v;
        }
        __syncthreads();
        s.med = uni(sh.bcd);
        __syncthreads();
    }
}

template <int NB, int TW>
__device__ __forceinline__ void scale_ref_pair(const AlignArgs& a, int level, RefShared<NB, TW>& sh) {
    constexpr int kRT = Geo<TW>::RT, kRW = TW;
    const int pair = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    PairState& S = a.state[pair];
    if (!S.active) return;
    const PairDesc& P = a.pairs[pair];
    const int nf = P.n_ref + P.n_kf;
    const uint32_t M = (uint32_t)nf * (uint32_t)a.area;
    const uint8_t* __restrict__ fvis = a.fvis + (int64_t)pair * a.max_f;
    uint32_t nrv = 0, ncv = 0;
    for (int f = tid; f < nf; f += kRT) {
        const uint8_t v = fvis[f];
        nrv += v & 1;
        ncv += v >> 1;
    }
    nrv = wave_sum_u(nrv);
    ncv = wave_sum_u(ncv);
    if (lane == 0) { sh.btot[wave] = nrv; sh.btot[kRW + wave] = ncv; }  // (btot is free until the first sweep)
    __syncthreads();
    nrv = 0; ncv = 0;
    for (int w = 0; w < kRW; ++w) { nrv += sh.btot[w]; ncv += sh.btot[kRW + w]; }
    __syncthreads();
    const uint32_t n = ncv * (uint32_t)a.area;
    double med = kDblMax, mad = 0.0;  // n == 0: every slot is DBL_MAX in the reference
    if (n > 0)
        ref_robust_scale<NB, TW, false>(a.scratch + (int64_t)pair * a.key_stride, sh, nullptr,
                                    a.sel + (int64_t)pair * a.sel_stride, a.sel_stride, M, n, med, mad);
    if (tid == 0) {
        double sigma = 1.482602218505602 * mad;
        if (sigma <= 2.220446049250313e-16) sigma = 2.220446049250313e-16;
        S.med = med;
        S.mad = mad;
        S.sigma = sigma;
        S.c = 4.6851 * sigma;
        S.n = n;
        S.n_ref_vis = nrv;
        S.scale_kernel = SVO_SCALE_K2R;
    }
}

constexpr uint32_t kSmallM = 64u * 2u * kBlk - 2u * kBlk;  // NB = 2 covers every segment of M <= 64512 slots

}  // namespace

// K2R: one workgroup per pair, two per CU (replaces align_scale_kernel when median_mode = SVO_MEDIAN_REFERENCE).
template <int NB, int TW>
__global__ void __launch_bounds__(Geo<TW>::RT, TW == 8 ? 2 : 1) __attribute__((amdgpu_waves_per_eu(4, 4)))
align_scale_ref_kernel(AlignArgs a, int level) {
    __shared__ RefShared<NB, TW> sh;
    scale_ref_pair<NB, TW>(a, level, sh);
}

// svo_debug_robust_scale: the same selection on an arbitrary residual vector (one workgroup)
template <int NB, int TW>
__global__ void __launch_bounds__(Geo<TW>::RT, TW == 8 ? 2 : 1) debug_robust_scale_kernel(const double* v, uint32_t M, uint32_t n, uint32_t* sel,
                                                                   int64_t sel_stride, double* out) {
    __shared__ RefShared<NB, TW> sh;
    __shared__ Diag dg;
    if (threadIdx.x == 0) {
        dg.cyc[0] = dg.cyc[1] = 0;
        dg.nblock[0] = dg.nblock[1] = dg.nlane[0] = dg.nlane[1] = dg.heap[0] = dg.heap[1] = 0;
        dg.nlog = 0;
        for (int i = 0; i < 16; ++i) dg.ph[i / 8][i % 8] = 0;
    }
    __syncthreads();
    double med = 0.0, mad = 0.0;
    ref_robust_scale<NB, TW, true>(v, sh, &dg, sel, sel_stride, M, n, med, mad);
    if (threadIdx.x == 0) {
        out[0] = med;
        out[1] = mad;
        for (int P = 0; P < 2; ++P) {
            out[2 + 4 * P] = (double)dg.cyc[P];
            out[3 + 4 * P] = (double)dg.nblock[P];
            out[4 + 4 * P] = (double)dg.nlane[P];
            out[5 + 4 * P] = (double)dg.heap[P];
        }
        for (int i = 0; i < 3 * kLogCap; ++i) out[10 + i] = i / 3 < (int)dg.nlog ? (double)dg.log[i / 3][i % 3] : -1.0;
        for (int i = 0; i < 16; ++i) out[190 + i] = (double)dg.ph[i / 8][i % 8];
    }
}

int ref_threads() { return Geo<8>::RT; }
// K2R scratch per pair, in u32: the segment (mp doubles), the mailbox (mp / 2), step records
int64_t ref_sel_stride(int64_t max_slots) {
    const int64_t mp = (max_slots + kBlk - 1) / kBlk * kBlk + kBlk;
    return 4 * mp;
}
// SVO_SCALE_IMPL (measurement knob, read once): 0 / unset (SVO_SCALE_AUTO) runs K2V wherever the vector fits
// its registers (<= refv_max_slots() slots; one pair per CU at 390 us per call against K2R's 643 us with two
// per CU: 110.5k vs 89.6k pairs/s at config 2), 1 forces K2R
int scale_impl() {
    static const int v = getenv("SVO_SCALE_IMPL") ? atoi(getenv("SVO_SCALE_IMPL")) : SVO_SCALE_AUTO;
    return v;
}
void launch_scale_ref(const AlignArgs& a, int level, hipStream_t s) {
    if (scale_impl() != SVO_SCALE_K2R && (int64_t)a.max_slots <= refv_max_slots()) {
        launch_scale_refv(a, level, s);
        return;
    }
    // a launch of at most 128 pairs (small batches, one pair per frame) gives each pair a whole CU
    const bool wide = a.n_pairs <= 128;
    const bool small = (int64_t)a.max_slots <= (int64_t)kSmallM;
    if (small && wide) hipLaunchKernelGGL((align_scale_ref_kernel<2, 16>), dim3(a.n_pairs), dim3(Geo<16>::RT), 0, s, a, level);
    else if (small) hipLaunchKernelGGL((align_scale_ref_kernel<2, 8>), dim3(a.n_pairs), dim3(Geo<8>::RT), 0, s, a, level);
    else if (wide) hipLaunchKernelGGL((align_scale_ref_kernel<17, 16>), dim3(a.n_pairs), dim3(Geo<16>::RT), 0, s, a, level);
    else hipLaunchKernelGGL((align_scale_ref_kernel<17, 8>), dim3(a.n_pairs), dim3(Geo<8>::RT), 0, s, a, level);
}
int launch_debug_robust_scale(const double* v, uint32_t M, uint32_t n, uint32_t* sel, int64_t sel_stride, int impl,
                              double* out, double* trace, uint32_t trcap, hipStream_t s, bool plain) {
    if (impl == SVO_SCALE_AUTO) impl = M <= (uint32_t)refv_max_slots() ? SVO_SCALE_K2V : SVO_SCALE_K2R;
    if (impl == SVO_SCALE_K2V) {
        if (M > (uint32_t)refv_max_slots()) return -1;
        launch_debug_robust_scale_v(v, M, n, reinterpret_cast<double*>(sel), out, trace, trcap, s, plain);
        return 0;
    }
    // (SVO_K2R_WAVES=16: the 16-wave instantiation, as small batches run it)
    static const bool w16 = getenv("SVO_K2R_WAVES") && atoi(getenv("SVO_K2R_WAVES")) == 16;
    if (M <= kSmallM) {
        if (w16) hipLaunchKernelGGL((debug_robust_scale_kernel<2, 16>), dim3(1), dim3(Geo<16>::RT), 0, s, v, M, n, sel, sel_stride, out);
        else hipLaunchKernelGGL((debug_robust_scale_kernel<2, 8>), dim3(1), dim3(Geo<8>::RT), 0, s, v, M, n, sel, sel_stride, out);
    } else {
        if (w16) hipLaunchKernelGGL((debug_robust_scale_kernel<17, 16>), dim3(1), dim3(Geo<16>::RT), 0, s, v, M, n, sel, sel_stride, out);
        else hipLaunchKernelGGL((debug_robust_scale_kernel<17, 8>), dim3(1), dim3(Geo<8>::RT), 0, s, v, M, n, sel, sel_stride, out);
    }
    return 0;
}

}  // namespace svo
