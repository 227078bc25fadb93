// align_ref.hip — K2R: the reference's robust scale bit for bit (median_mode SVO_MEDIAN_REFERENCE).
//
// Optimizer::tukeyWeighting (src/optimizer.cpp:485-514) takes sigma = 1.482602218505602 * MAD with
// algorithm::computeMedian (src/algorithm.cpp:834-853) on the FULL residual vector (n_features * patch^2
// slots in feature-major order, invisible slots = DBL_MAX): std::nth_element(vec, vec + n/2), then, for an
// even total length, (vec[n/2 - 1] + vec[n/2]) / 2 — where vec[n/2 - 1] is whatever libstdc++'s
// introselect left there, not always the (n/2 - 1)-th order statistic.  The MAD is the
// same call on |r_i - median| in the original order (:855-865).
//
// K2R re-runs libstdc++'s introselect (stl_algo.h __introselect, GCC 11) on the device, one 1024-thread
// workgroup per pair.  Each partition round is evaluated in the parallel form that
// tests/cpp/introselect_model.cpp derives and checks against std::nth_element:
//   median of three (first+1, first+S/2, last-1) moved to first, pivot p;
//   GE = positions in [first+1, last) with !(a < p), LE = positions in [first, last) with !(p < a);
//   the Hoare loop swaps the k-th GE from the left with the k-th LE from the right for k <= Ks,
//   Ks = max over split points t of min(#GE before t, #LE from t on), and returns
//   cut = min(L_{Ks+1}, R_{Ks}).
// so a round is: the pivot (one lane), a counting sweep (ballots), a block scan, the crossing (one wave),
// a ranking sweep (L_{Ks+1}, R_{Ks}, the swap partners), and the swaps.  The depth limit falls back to the
// restated heap select (one lane; only adversarial inputs reach it), the last <= 3 values are sorted.
// vec[n/2 - 1] is recorded at the round whose cut lands exactly on n/2 (afterwards that slot is never
// touched again), or read after the final sort.
//
// Elements are (32-bit residual key of svo_wave.h res_key32, slot id).  Keys order residuals exactly
// except inside one 2^-22 grid cell; the few comparisons they cannot settle use the exact residual,
// recomputed from the images by slot id (the same per-sample arithmetic K1's keys come from).  The MAD
// pass compares |r - median| through the keys' residual intervals and four key thresholds per pivot.
// Round 1 streams K1's feature-major keys (16-B loads); the surviving segment goes to LDS (keys + 16-bit
// ids when the vector has <= 65536 slots) when it fits, else to the pair's global scratch (sel) until it
// does.  A round classifies every element once, keeping per-64-position-step GE / LE ballots in the
// registers of the wave that owns the step; the scans, the crossing, L_{Ks+1} / R_{Ks} and each swap's
// partners come from those records.  Segments of <= 64 steps run on one wave without barriers.
//
// Code size matters: the pass (median / MAD) and the segment's storage are runtime values, each phase is
// compiled once (only the innermost loops are specialised), so the kernel's hot code stays inside the
// instruction cache.
#include "svo_internal.h"
#include "svo_math.h"
#include "svo_wave.h"

namespace svo {

namespace {

constexpr int kRT = 512;               // threads per pair
constexpr int kRW = kRT / 64;          // waves
constexpr int kMeta = 1024;            // LDS step records (64 positions each): segments up to 65536
constexpr int kBatch = 4;
constexpr uint32_t kWaveSteps = 8;     // segments of <= 8 steps run on one wave (block rounds above)              // loads a lane issues before using any (copies, swaps)
constexpr uint32_t kNone = 0xFFFFFFFFu;
constexpr double kDblMax = 1.7976931348623157e308;

struct El {
    uint32_t key, id;
};

struct Pivot {
    El e;
    El f0;                   // the element the median of three displaced from `first` (now at ch)
    uint32_t ch;             // position the median of three came from
    int inv;                 // pass 1: the pivot is DBL_MAX (an invisible slot)
    double plo, phi;         // pass 1: |r - med| interval of the pivot (equal: exact)
    int64_t kA, kB, kC, kD;  // pass 1: key-grid thresholds (see classify)
    // branch-free fast classification (see fast_cls): the pivot's key, and for pass 1 the key ranges
    // [tA, tB] (certainly |r - med| < plo), <= tC or >= tD (certainly > phi), the class of an invisible key
    uint32_t tA, tB, tC, tD, inv_c;
};

template <typename Id>
struct RefShared {
    static constexpr int kCap = sizeof(Id) == 2 ? 16384 : 12288;  // LDS segment capacity (elements)
    alignas(16) uint32_t key[kCap + 64];     // the segment, from position `base` (+64: whole-step reads)
    Id id[kCap];
    uint16_t lp[kCap / 2], rp[kCap / 2];     // L_k, R_k - b0 for k <= Ks (LDS rounds)
    uint64_t mge[kMeta], mle[kMeta];         // per 64-position step: GE / LE ballots
    uint32_t gpre[kMeta], lsuf[kMeta];       // per step: #GE before it, #LE from its first position on
    uint32_t wsum[kRW][2];
    Pivot piv;
    uint32_t ks, cut_l, cut_r, l_ks;
    uint32_t bc_first, bc_last, bc_depth, bc_rec;
    El lo_el, fin[3];
    uint32_t wlog[22][3];  // diagnostics: per wave round (both passes): steps, sweep cycles, round cycles
    uint32_t nwlog;
    uint32_t blog[40][3];  // diagnostics: per block round: segment size, where, cycles
    uint32_t nblog;
    uint64_t stamp[32];  // diagnostics (svo_debug_robust_scale): per pass: cycles of round 1, of the rest,
                         // block rounds, wave rounds; [8..] cycles per phase of block rounds; [28..] exact calls
};

// where the current segment lives
enum { kSrc = 0, kGlb = 1, kLds = 2 };

// ---- element sources: round-1 keys in the reference's order, and the exact residual of a slot
struct ImgSrc {  // production: K1's keys and the images
    using KeyBase = const uint32_t*;
    static __device__ __forceinline__ uint32_t key_at(KeyBase kb, uint32_t p) { return kb[p]; }
    const uint32_t* keys;   // pair's feature-major keys: slot f * area + k (padded)
    const double* px;       // pair's feature pixels (level 0)
    const double* cproj;    // pair's projections into the cur level (K1)
    const uint8_t *rplane, *kplane, *cplane;
    int W, area, side, half, n_ref;
    double scale;
    __device__ __forceinline__ uint32_t key(uint32_t p) const { return keys[p]; }
    __device__ __forceinline__ KeyBase kbase() const { return keys; }
    // r = bilerpD(I_cur, cu + kx, cv + ky) - bilerpD(I_ref, u + kx, v + ky)  (src/image_alignment.cpp:351-359)
    __device__ double r(uint32_t s) const {
        const int f = (int)(s / (uint32_t)area), k = (int)s - f * area;
        const int ky = k / side, kx = k - ky * side;
        const double ur = px[2 * f] * scale, vr = px[2 * f + 1] * scale;
        const double cu = cproj[2 * f], cv = cproj[2 * f + 1];
        const double T = bilinear_d(f < n_ref ? rplane : kplane, W, ur + (double)(kx - half), vr + (double)(ky - half));
        const double I = bilinear_d(cplane, W, cu + (double)(kx - half), cv + (double)(ky - half));
        return I - T;
    }
};
struct ArrSrc {  // svo_debug_robust_scale: an arbitrary residual vector (>= DBL_MAX = invisible), its keys
    using KeyBase = const uint32_t*;
    static __device__ __forceinline__ uint32_t key_at(KeyBase kb, uint32_t p) { return kb[p]; }
    const double* v;
    const uint32_t* keys;
    __device__ __forceinline__ uint32_t key(uint32_t p) const { return keys[p]; }
    __device__ __forceinline__ KeyBase kbase() const { return keys; }
    __device__ __forceinline__ double r(uint32_t s) const { return v[s]; }
};

__device__ __forceinline__ int lg2(uint32_t n) { return 31 - __builtin_clz(n); }
__device__ __forceinline__ uint64_t low_mask(uint32_t b) { return b >= 64 ? ~0ull : ((1ull << b) - 1ull); }
__device__ __forceinline__ uint64_t lane_read_u64(uint64_t v, int l) {
    return ((uint64_t)lane_read((uint32_t)(v >> 32), l) << 32) | lane_read((uint32_t)v, l);
}
// position of the j-th (0-based) set bit of m
__device__ __forceinline__ uint32_t select_bit(uint64_t m, uint32_t j) {
    uint32_t pos = 0;
#pragma unroll
    for (int w = 32; w >= 1; w >>= 1) {
        const uint32_t c = (uint32_t)__popcll(m & ((1ull << w) - 1ull));
        if (j >= c) { j -= c; m >>= w; pos += (uint32_t)w; }
    }
    return pos;
}

// ---- values and comparisons (P: 0 = the residual, 1 = |residual - med|)
__device__ __forceinline__ void d_interval(uint32_t k, double med, double& lo, double& hi) {  // |r - med| over the key's cell
    const double rl = key_r(k), rh = (k & 1u) ? rl + kKeyStep : rl;
    if (rh <= med) { lo = med - rh; hi = med - rl; }
    else if (rl >= med) { lo = rl - med; hi = rh - med; }
    else { lo = 0.0; hi = fmax(med - rl, rh - med); }
}
template <class Src>
__device__ __forceinline__ double value(const Src* src, int P, double med, El e) {  // the reference's vector entry
    if (e.key == kKeyInvisible) return kDblMax;
    const double r = (e.key & 1u) ? src->r(e.id) : key_r(e.key);
    return P == 0 ? r : fabs(r - med);
}
// value(a) < value(b), exact (the keys decide almost always; the images only inside one key cell)
template <class Src>
__device__ __attribute__((noinline)) bool less_slow(const Src* src, int P, double med, El a, El b) {
    return value(src, P, med, a) < value(src, P, med, b);
}
template <class Src>
__device__ __forceinline__ bool less(const Src* src, int P, double med, El a, El b) {
    if (P == 0) {
        if (a.key != b.key) return a.key < b.key;
        if (a.key == kKeyInvisible || !(a.key & 1u)) return false;
    } else {
        if (a.key == kKeyInvisible) return false;
        if (b.key == kKeyInvisible) return true;
        double alo, ahi, blo, bhi;
        d_interval(a.key, med, alo, ahi);
        d_interval(b.key, med, blo, bhi);
        if (ahi < blo) return true;
        if (alo >= bhi) return false;
    }
    return less_slow(src, P, med, a, b);
}
// (ge, le) of an element whose key missed the fast tests: the cell's interval, then the exact values
template <class Src>
__device__ __attribute__((noinline)) uint32_t classify_slow(const Src* src, int P, double med, uint32_t k, uint32_t id,
                                                           El pe, double plo, double phi, uint64_t* counter) {
    if (P == 1) {
        double lo, hi;
        d_interval(k, med, lo, hi);
        if (hi < plo) return 2u;
        if (lo > phi) return 1u;
    }
    if (counter) atomicAdd((unsigned long long*)counter, 1ull);  // diagnostics
    const double v = value(src, P, med, El{k, id}), p = value(src, P, med, pe);
    return (!(v < p) ? 1u : 0u) | (!(p < v) ? 2u : 0u);
}

// ---- heap select (depth limit), one lane: stl_heap.h __adjust_heap / __push_heap / __make_heap /
// __pop_heap and stl_algo.h __heap_select restated over positions first + i, then the swap of first and
// nth (tests/cpp/introselect_model.cpp checks the restatement).  Only adversarial inputs reach it; a free
// function of plain values, so that the selection state never needs an address.
template <class Src, typename Id>
struct HeapView {
    const Src* src;
    RefShared<Id>* sh;
    uint32_t* gkey;
    uint32_t* gid;
    uint32_t first, base;
    int where, P;
    double med;
    __device__ El get(uint32_t i) const {
        const uint32_t p = first + i;
        if (where == kLds) return El{sh->key[p - base], (uint32_t)sh->id[p - base]};
        if (where == kGlb) return El{gkey[p], gid[p]};
        return El{src->key(p), p};
    }
    __device__ void put(uint32_t i, El e) const {
        const uint32_t p = first + i;
        if (where == kLds) { sh->key[p - base] = e.key; sh->id[p - base] = (Id)e.id; }
        else if (where == kGlb) { gkey[p] = e.key; gid[p] = e.id; }
    }
    __device__ bool lt(El a, El b) const { return less(src, P, med, a, b); }
};
template <class Src, typename Id>
__device__ __attribute__((noinline)) void heap_select_fn(HeapView<Src, Id> h, uint32_t middle, uint32_t len, uint32_t nth_rel) {
    auto push_heap = [&](uint32_t hole, uint32_t top, El value) {
        uint32_t parent = (hole - 1) / 2;
        while (hole > top && h.lt(h.get(parent), value)) {
            h.put(hole, h.get(parent));
            hole = parent;
            parent = (hole - 1) / 2;
        }
        h.put(hole, value);
    };
    auto adjust_heap = [&](uint32_t hole, uint32_t n, El value) {
        const uint32_t top = hole;
        uint32_t second = hole;
        while (n >= 1 && second < (n - 1) / 2) {
            second = 2 * (second + 1);
            if (h.lt(h.get(second), h.get(second - 1))) second--;
            h.put(hole, h.get(second));
            hole = second;
        }
        if ((n & 1u) == 0 && second == (n - 2) / 2) {
            second = 2 * (second + 1);
            h.put(hole, h.get(second - 1));
            hole = second - 1;
        }
        push_heap(hole, top, value);
    };
    if (middle >= 2) {
        uint32_t parent = (middle - 2) / 2;
        while (true) {
            adjust_heap(parent, middle, h.get(parent));
            if (parent == 0) break;
            parent--;
        }
    }
    for (uint32_t i = middle; i < len; ++i)
        if (h.lt(h.get(i), h.get(0))) {
            const El v = h.get(i);
            h.put(i, h.get(0));
            adjust_heap(0, middle, v);
        }
    const El f0 = h.get(0), n0 = h.get(nth_rel);  // std::iter_swap(first, nth)
    h.put(0, n0);
    h.put(nth_rel, f0);
}

// block-uniform values read from LDS, moved to scalar registers: the compiler cannot prove them uniform,
// and control flow on a vector value becomes exec-mask code (every loop over steps, every branch on the
// round's state)
__device__ __forceinline__ uint32_t uni(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t uni(uint64_t v) { return ((uint64_t)uni((uint32_t)(v >> 32)) << 32) | uni((uint32_t)v); }
__device__ __forceinline__ int64_t uni(int64_t v) { return (int64_t)uni((uint64_t)v); }
__device__ __forceinline__ double uni(double v) { return __builtin_bit_cast(double, uni(__builtin_bit_cast(uint64_t, v))); }
__device__ __forceinline__ El uni(El e) { return El{uni(e.key), uni(e.id)}; }
__device__ __forceinline__ Pivot uni(const Pivot& p) {
    Pivot q;
    q.e = uni(p.e); q.f0 = uni(p.f0); q.ch = uni(p.ch); q.inv = uni(p.inv);
    q.plo = uni(p.plo); q.phi = uni(p.phi);
    q.kA = uni(p.kA); q.kB = uni(p.kB); q.kC = uni(p.kC); q.kD = uni(p.kD);
    q.tA = uni(p.tA); q.tB = uni(p.tB); q.tC = uni(p.tC); q.tD = uni(p.tD); q.inv_c = uni(p.inv_c);
    return q;
}

// kSt: diagnostics (svo_debug_robust_scale): clock stamps per phase / round; compiled out of the product
template <class Src, typename Id, bool kSt>
struct RefSel {
    using Shared = RefShared<Id>;
    static constexpr int kCap = Shared::kCap;
    static constexpr int R = sizeof(Id) == 2 ? 2 : 16;  // step records per lane (segments up to 64 R steps / wave)
    const Src* src;   // the source, kept in LDS (the slow paths take this pointer, never a copy)
    Shared& sh;
    typename Src::KeyBase kb;  // round-1 keys (inline path)
    uint32_t* gkey;   // pair's global segment keys / ids (absolute positions)
    uint32_t* gid;
    uint32_t* glp;    // swap partners L_k / R_k of the global and copy rounds
    uint32_t* grp;
    uint64_t* gmge;   // step records of segments past kMeta steps (R > 1)
    uint64_t* gmle;
    uint32_t* ggpre;  // their per-step prefix counts
    uint32_t* glsuf;
    uint32_t M, nth;
    int tid, lane, wave;
    int P;            // the pass: 0 median, 1 MAD
    double med;       // pass 1
    // block-uniform state
    uint32_t first, last, base;
    int where, depth, rec;
    El lo_el;
    Pivot pv;

    // ---------------------------------------------------------------- storage (runtime `where`)
    __device__ __forceinline__ El get(uint32_t p) const {
        if (where == kLds) return El{sh.key[p - base], (uint32_t)sh.id[p - base]};
        if (where == kGlb) return El{gkey[p], gid[p]};
        return El{Src::key_at(kb, p), p};
    }
    __device__ __forceinline__ void put(uint32_t p, El e) {
        if (where == kLds) { sh.key[p - base] = e.key; sh.id[p - base] = (Id)e.id; }
        else if (where == kGlb) { gkey[p] = e.key; gid[p] = e.id; }
    }
    // the segment after the median-of-three swap (first <-> ch), before it is stored
    __device__ __forceinline__ El elp(uint32_t p) const {
        if (p == first) return pv.e;
        if (p == pv.ch) return pv.f0;
        return get(p);
    }
    __device__ __forceinline__ uint32_t idp(uint32_t p) const { return elp(p).id; }

    // (ge, le) = (!(a < p), !(p < a)) as bits 0, 1 for the element of key k at position p
    __device__ __forceinline__ uint32_t classify(uint32_t k, uint32_t p) const {
        if (P == 0) {
            if (k != pv.e.key) return k < pv.e.key ? 2u : 1u;
            if (k == kKeyInvisible || !(k & 1u)) return 3u;
        } else {
            if (pv.inv) return k == kKeyInvisible ? 3u : 2u;
            if (k == kKeyInvisible) return 1u;
            const int64_t g = (int64_t)(k >> 1);
            // |r - med| < plo for the whole cell: r two grid steps inside (med - plo, med + plo)
            if (g >= pv.kA + 2 && g <= pv.kB - 2) return 2u;
            // |r - med| > phi for the whole cell: r two grid steps outside [med - phi, med + phi]
            if (g <= pv.kC - 2 || g >= pv.kD + 2) return 1u;
        }
        return classify_slow(src, P, med, k, idp(p), pv.e, pv.plo, pv.phi, kSt ? &sh.stamp[28 + P] : nullptr);
    }
    // the pivot: std::__move_median_to_first(first, first + 1, first + S/2, last - 1) and the pass-1
    // interval / thresholds of the chosen element (uniform; every caller lane computes the same)
    __device__ __forceinline__ void choose_pivot() {
        const uint32_t S = last - first, A = first + 1, B = first + S / 2, C = last - 1;
        const El a = get(A), b = get(B), c = get(C);
        uint32_t ch;
        El e;
        if (less(src, P, med, a, b)) {
            if (less(src, P, med, b, c)) { ch = B; e = b; }
            else if (less(src, P, med, a, c)) { ch = C; e = c; }
            else { ch = A; e = a; }
        } else if (less(src, P, med, a, c)) { ch = A; e = a; }
        else if (less(src, P, med, b, c)) { ch = C; e = c; }
        else { ch = B; e = b; }
        pv.f0 = get(first);
        pv.ch = ch;
        pivot_fields(e);
    }
    // the pivot's pass-1 interval and key thresholds (uniform; every caller lane computes the same)
    __device__ __forceinline__ void pivot_fields(El e) {
        pv.e = e;
        pv.inv = e.key == kKeyInvisible;
        pv.plo = pv.phi = 0.0;
        pv.kA = pv.kB = pv.kC = pv.kD = 0;
        // pass 1, as key ranges: visible keys are > 2^29 (|r| <= 255), so tC = 0 / tD = ~0 are empty ranges
        pv.tA = 1; pv.tB = 0; pv.tC = 0; pv.tD = kKeyInvisible;
        pv.inv_c = 1u;  // an invisible slot is DBL_MAX: greater than a visible pivot
        if (P == 1 && pv.inv) {
            pv.tA = 0; pv.tB = kKeyInvisible - 1; pv.inv_c = 3u;  // every visible slot is less; DBL_MAX equal
        } else if (P == 1) {
            d_interval(e.key, med, pv.plo, pv.phi);
            pv.kA = key_grid(med - pv.plo);
            pv.kB = key_grid(med + pv.plo);
            pv.kC = key_grid(med - pv.phi);
            pv.kD = key_grid(med + pv.phi);
            const int64_t a0 = 2 * (pv.kA + 2), b0 = 2 * (pv.kB - 2) + 1, c0 = 2 * (pv.kC - 2) + 1, d0 = 2 * (pv.kD + 2);
            if (a0 <= b0 && b0 >= 0 && a0 <= (int64_t)kKeyInvisible - 1) {
                pv.tA = (uint32_t)(a0 < 0 ? 0 : a0);
                pv.tB = (uint32_t)(b0 > (int64_t)kKeyInvisible - 1 ? (int64_t)kKeyInvisible - 1 : b0);
            }
            if (c0 >= 0) pv.tC = (uint32_t)(c0 > (int64_t)kKeyInvisible - 1 ? (int64_t)kKeyInvisible - 1 : c0);
            if (d0 <= (int64_t)kKeyInvisible - 1) pv.tD = (uint32_t)(d0 < 0 ? 0 : d0);
        }
    }
    // ---------------------------------------------------------------- classification sweep
    // A step is 64 positions, lane = position.  Its GE / LE masks come straight out of vector compares
    // (the compare's lane mask IS the ballot): pass 0 ge = (k >= pk), le = (k <= pk); pass 1 from the key
    // ranges of choose_pivot (lt = [tA, tB], gt = <= tC or >= tD; ge = ~lt, le = ~gt).  Only keys the
    // compares cannot settle (same inexact cell as the pivot, pass-1 boundary cells) take classify_slow
    // under one wave-uniform test.  The masks go to the lane that owns the step (writelane), so a wave
    // holds the records of up to 64 RR steps in registers: lane j of row r = step s0 + 64 r + j.
    // Positions outside (first, last), `first` itself (the pivot: LE only) and ch (holding f0 after the
    // median-of-three swap) are fixed afterwards, per record (fix_rows).
    // G: the segment is in global memory (gk = the read-only round-1 keys or the pair's scratch), else LDS.
    // One instantiation serves both global kinds: code size is what limits the serial parts (I-cache).
    template <bool G>
    __device__ __forceinline__ uint32_t load_key(const uint32_t* gk, uint32_t p) const {
        if (G) return gk[p];
        return sh.key[p - base];
    }
    template <bool G>
    __device__ __forceinline__ uint32_t load_id(uint32_t p) const {
        if (G) return where == kSrc ? p : gid[p];
        return (uint32_t)sh.id[p - base];
    }
    // bits i with a <= sp + i < b
    static __device__ __forceinline__ uint64_t range_mask(uint32_t sp, uint32_t a, uint32_t b) {
        const uint32_t lo = a > sp ? (a - sp < 64u ? a - sp : 64u) : 0u;
        const uint32_t hi = b > sp ? (b - sp < 64u ? b - sp : 64u) : 0u;
        return low_mask(hi) & ~low_mask(lo);
    }
    template <bool G>
    __device__ __forceinline__ void slow_fix(uint32_t sp, uint32_t k, uint64_t sl, uint64_t& ge, uint64_t& le) const {
        sl &= range_mask(sp, first + 1, last);
        const bool me = (sl >> lane) & 1ull;
        uint32_t c = 0;
        if (me) c = classify_slow(src, P, med, k, load_id<G>(sp + (uint32_t)lane), pv.e, pv.plo, pv.phi, kSt ? &sh.stamp[28 + P] : nullptr);
        ge = (ge & ~sl) | __ballot(me && (c & 1u));
        le = (le & ~sl) | __ballot(me && (c & 2u));
    }
    // a step's masks from the compares; sl = positions the keys cannot settle
    struct Thr {
        uint32_t pk, tA, tB, tC, tD;
        bool pslow, pinv;
    };
    __device__ __forceinline__ Thr thresholds() const {
        Thr t;
        t.pk = uni(pv.e.key);
        t.tA = uni(pv.tA); t.tB = uni(pv.tB); t.tC = uni(pv.tC); t.tD = uni(pv.tD);
        t.pslow = (t.pk & 1u) && t.pk != kKeyInvisible;  // pass 0: equal keys need the exact values
        t.pinv = uni(pv.inv) != 0;
        return t;
    }
    template <int PP>
    static __device__ __forceinline__ void step_masks(const Thr& t, uint32_t k, uint64_t& ge, uint64_t& le, uint64_t& sl) {
        if (PP == 0) {
            ge = __ballot(k >= t.pk);
            le = __ballot(k <= t.pk);
            sl = t.pslow ? __ballot(k == t.pk) : 0ull;
        } else if (t.pinv) {  // pivot DBL_MAX: every visible slot is less, DBL_MAX equal
            ge = __ballot(k == kKeyInvisible);
            le = ~0ull;
            sl = 0ull;
        } else {
            const uint64_t lt = __ballot(k >= t.tA) & __ballot(k <= t.tB);
            const uint64_t gt = __ballot(k <= t.tC) | __ballot(k >= t.tD);
            ge = ~lt;
            le = ~gt;
            sl = ~(lt | gt);
        }
    }
    template <int RR, bool G, int PP>
    __device__ __forceinline__ void sweep_rows(uint32_t b0, uint32_t s0, uint32_t n, uint64_t (&mg)[RR], uint64_t (&ml)[RR]) const {
        b0 = uni(b0); s0 = uni(s0); n = uni(n);  // scalar loop control (see uni)
        const uint32_t* const gk = where == kSrc ? kb : gkey;
        const Thr t = thresholds();
#pragma unroll
        for (int r = 0; r < RR; ++r) {
            uint32_t g0 = 0, g1 = 0, l0 = 0, l1 = 0;
            const uint32_t nr = n > 64u * r ? (n - 64u * r < 64u ? n - 64u * r : 64u) : 0u;
            const uint32_t sr = s0 + 64u * r;
            for (uint32_t j0 = 0; j0 < nr; j0 += 8) {
                uint32_t kv[8];
#pragma unroll
                for (int b = 0; b < 8; ++b) kv[b] = load_key<G>(gk, b0 + 64u * (sr + j0 + (uint32_t)b) + (uint32_t)lane);
                uint64_t any = 0;
#pragma unroll
                for (int b = 0; b < 8; ++b) {
                    const uint32_t j = j0 + (uint32_t)b;
                    if (j >= nr) break;  // wave-uniform
                    uint64_t ge, le, sl;
                    step_masks<PP>(t, kv[b], ge, le, sl);
                    any |= sl;
                    g0 = lane_write(g0, (uint32_t)ge, j);
                    g1 = lane_write(g1, (uint32_t)(ge >> 32), j);
                    l0 = lane_write(l0, (uint32_t)le, j);
                    l1 = lane_write(l1, (uint32_t)(le >> 32), j);
                }
                if (any) {  // rare: redo the batch's unsettled steps exactly (one copy of the slow path)
                    const uint32_t je = j0 + 8u < nr ? j0 + 8u : nr;
#pragma unroll 1
                    for (uint32_t j = j0; j < je; ++j) {
                        const uint32_t sp = b0 + 64u * (sr + j);
                        const uint32_t k = load_key<G>(gk, sp + (uint32_t)lane);
                        uint64_t ge, le, sl;
                        step_masks<PP>(t, k, ge, le, sl);
                        if (sl) {
                            slow_fix<G>(sp, k, sl, ge, le);
                            g0 = lane_write(g0, (uint32_t)ge, j);
                            g1 = lane_write(g1, (uint32_t)(ge >> 32), j);
                            l0 = lane_write(l0, (uint32_t)le, j);
                            l1 = lane_write(l1, (uint32_t)(le >> 32), j);
                        }
                    }
                }
            }
            mg[r] = ((uint64_t)g1 << 32) | g0;
            ml[r] = ((uint64_t)l1 << 32) | l0;
        }
    }
    template <int RR>
    __device__ __forceinline__ void sweep_rows(uint32_t b0, uint32_t s0, uint32_t n, uint64_t (&mg)[RR], uint64_t (&ml)[RR]) const {
        if (P == 0) {
            if (where == kLds) sweep_rows<RR, false, 0>(b0, s0, n, mg, ml);
            else sweep_rows<RR, true, 0>(b0, s0, n, mg, ml);
        } else {
            if (where == kLds) sweep_rows<RR, false, 1>(b0, s0, n, mg, ml);
            else sweep_rows<RR, true, 1>(b0, s0, n, mg, ml);
        }
    }
    // the records' edge fixes (lanes holding a step of this wave only): GE in (first, last), LE in
    // [first, last) with `first` LE, ch classified as f0 (f0c)
    template <int RR>
    __device__ __forceinline__ void fix_rows(uint32_t b0, uint32_t s0, uint32_t n, uint32_t f0c, uint64_t (&mg)[RR], uint64_t (&ml)[RR]) const {
#pragma unroll
        for (int r = 0; r < RR; ++r) {
            const uint32_t j = 64u * r + (uint32_t)lane;
            const uint32_t sp = b0 + 64u * (s0 + j);
            if (j < n) {
                mg[r] &= range_mask(sp, first + 1, last);
                ml[r] &= range_mask(sp, first, last);
                if (first >= sp && first < sp + 64u) ml[r] |= 1ull << (first - sp);
                if (pv.ch >= sp && pv.ch < sp + 64u) {
                    const uint64_t bit = 1ull << (pv.ch - sp);
                    mg[r] = (mg[r] & ~bit) | ((f0c & 1u) ? bit : 0ull);
                    ml[r] = (ml[r] & ~bit) | ((f0c & 2u) ? bit : 0ull);
                }
            } else {
                mg[r] = 0ull;
                ml[r] = 0ull;
            }
        }
    }
    // ---------------------------------------------------------------- swap partners, lane = position
    // Over the steps a wave holds in registers (lane j of row r = step s0 + 64 r + j: records mg / ml and
    // the prefix counts gp = #GE before the step, ls = #LE from its start on), read per step with readlane:
    // the GE of rank k = gp + (GE bits below) + 1 is L_k, the LE of right-rank k = ls - (LE bits below) is
    // R_k; k <= Ks go to the lists, L_{Ks+1} / L_{Ks} / R_{Ks} to the shared scalars (one position holds
    // each rank, so one lane writes each).  A step whose ranks all exceed Ks + 1 is skipped (uniform test):
    // left of the crossing only the GE part runs, right of it only the LE part.
    template <int RR, bool LL>
    __device__ __forceinline__ void partners_t(uint32_t b0, uint32_t s0, uint32_t n, uint32_t ks, const uint64_t (&mg)[RR],
                                               const uint64_t (&ml)[RR], const uint32_t (&gp)[RR], const uint32_t (&ls)[RR],
                                               uint16_t* lpl, uint16_t* rpl) {
        b0 = uni(b0); s0 = uni(s0); n = uni(n); ks = uni(ks);
        const uint64_t mybit = 1ull << lane;
        auto put_l = [&](uint32_t k, uint32_t pos) {
            if (LL) lpl[k - 1] = (uint16_t)(pos - b0);
            else glp[k - 1] = pos;
        };
        auto put_r = [&](uint32_t k, uint32_t pos) {
            if (LL) rpl[k - 1] = (uint16_t)(pos - b0);
            else grp[k - 1] = pos;
        };
#pragma unroll
        for (int r = 0; r < RR; ++r) {
            const uint32_t nr = n > 64u * r ? (n - 64u * r < 64u ? n - 64u * r : 64u) : 0u;
            for (uint32_t j = 0; j < nr; ++j) {
                const uint32_t g = lane_read(gp[r], (int)j), l = lane_read(ls[r], (int)j);
                const uint32_t pos = b0 + 64u * (s0 + 64u * r + j) + (uint32_t)lane;
                if (g <= ks) {  // GE ranks g + 1 .. g + popc(a) reach Ks + 1
                    const uint64_t a = lane_read_u64(mg[r], (int)j);
                    const uint32_t k = __builtin_amdgcn_mbcnt_hi((uint32_t)(a >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)a, g + 1u));
                    if (g + (uint32_t)__popcll(a) < ks) {  // every rank < Ks: plain compaction
                        if (a & mybit) put_l(k, pos);
                    } else if (a & mybit) {
                        if (k <= ks) put_l(k, pos);
                        if (k == ks + 1u) sh.cut_l = pos;
                        if (k == ks) sh.l_ks = pos;
                    }
                }
                const uint64_t bb = lane_read_u64(ml[r], (int)j);
                if (l - (uint32_t)__popcll(bb) < ks) {  // LE right-ranks l - popc + 1 .. l reach Ks
                    const uint32_t k = l - lanes_below(bb);
                    if (l < ks) {
                        if (bb & mybit) put_r(k, pos);
                    } else if ((bb & mybit) && k <= ks) {
                        put_r(k, pos);
                        if (k == ks) sh.cut_r = pos;
                    }
                }
            }
        }
    }
    template <int RR>
    __device__ __forceinline__ void partners(uint32_t b0, uint32_t s0, uint32_t n, uint32_t ks, const uint64_t (&mg)[RR],
                                             const uint64_t (&ml)[RR], const uint32_t (&gp)[RR], const uint32_t (&ls)[RR],
                                             bool lds_lists, uint16_t* lpl, uint16_t* rpl) {
        if (lds_lists) partners_t<RR, true>(b0, s0, n, ks, mg, ml, gp, ls, lpl, rpl);
        else partners_t<RR, false>(b0, s0, n, ks, mg, ml, gp, ls, lpl, rpl);
    }

    // ---------------------------------------------------------------- one block round (large segments)
    // Steps are 64 positions from b0 = first & ~63; wave w owns the steps [w spw, (w + 1) spw) with
    // spw = ceil(steps / 16) <= 64 R, lane l holding steps w spw + 64 r + l in registers: GE / LE ballots,
    // in-wave prefix sums, the GE count before and the LE count from each step.  Wave 0 chooses the pivot
    // and finds the crossing; barriers after the pivot, the sweep, the crossing, the partner lists and the
    // swaps.
    __device__ __forceinline__ void round() {
        first = uni(first); last = uni(last);
        const uint32_t b0 = first & ~63u, ns = (last - b0 + 63) / 64;
        const uint32_t spw = (ns + kRW - 1) / kRW;
        uint64_t* const mge = R <= 2 ? sh.mge : gmge;
        uint64_t* const mle = R <= 2 ? sh.mle : gmle;
        uint32_t* const mgp = R <= 2 ? sh.gpre : ggpre;
        uint32_t* const mls = R <= 2 ? sh.lsuf : glsuf;
        uint64_t tp = kSt ? clock64() : 0;
        auto phase = [&](int i) {
            if (kSt && tid == 0) { const uint64_t t = clock64(); sh.stamp[8 + 5 * where + i] += t - tp; tp = t; }
        };
        // every wave chooses the same pivot (3 reads and compares; no barrier, no broadcast)
        choose_pivot();
        pv = uni(pv);
        if (tid == 0) { sh.cut_l = kNone; sh.cut_r = kNone; sh.l_ks = kNone; }  // read after two barriers
        phase(0);
        // ---- classification sweep of the wave's steps, records in registers, then to the step arrays
        const uint32_t ws0 = (uint32_t)wave * spw;
        const uint32_t wsn = ws0 >= ns ? 0u : (ns - ws0 < spw ? ns - ws0 : spw);
        const uint32_t f0c = classify(pv.f0.key, pv.ch);
        uint64_t mg[R], ml[R];
        sweep_rows<R>(b0, ws0, wsn, mg, ml);
        fix_rows<R>(b0, ws0, wsn, f0c, mg, ml);
        uint32_t gex[R], lex[R], gw = 0, lw = 0;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const uint32_t j = 64 * (uint32_t)r + (uint32_t)lane;
            if (j < wsn) { mge[ws0 + j] = mg[r]; mle[ws0 + j] = ml[r]; }
            const uint32_t cg = (uint32_t)__popcll(mg[r]), cl = (uint32_t)__popcll(ml[r]);
            const uint32_t gi = wave_incl_scan(cg), li = wave_incl_scan(cl);
            gex[r] = gw + gi - cg;
            lex[r] = lw + li - cl;
            gw += lane_read(gi, 63);
            lw += lane_read(li, 63);
        }
        if (lane == 0) { sh.wsum[wave][0] = gw; sh.wsum[wave][1] = lw; }
        if (R > 2) __threadfence_block();  // global step records before the barrier
        __syncthreads();
        phase(1);
        // ---- wave prefixes (lane i < kRW holds wave i's totals), the per-step prefix arrays; the crossing t*
        // (first split with G >= Lc): its wave, its step, its bit, Ks = max(G(t*-1), Lc(t*)), found by wave 0
        const uint32_t wg = lane < kRW ? sh.wsum[lane][0] : 0u, wl = lane < kRW ? sh.wsum[lane][1] : 0u;
        const uint32_t wgi = wave_incl_scan(wg), wli = wave_incl_scan(wl);
        const uint32_t lt = lane_read(wli, 63);
        const uint32_t gb = lane_read(wgi - wg, wave), lb = lane_read(wli - wl, wave);
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const uint32_t j = 64 * (uint32_t)r + (uint32_t)lane;
            if (j < wsn) { mgp[ws0 + j] = gb + gex[r]; mls[ws0 + j] = lt - lb - lex[r]; }
        }
        uint32_t ks;
        {  // every wave finds the same crossing (no barrier, no broadcast)
            const uint32_t g_start = wgi - wg, l_start = lt - (wli - wl);
            const uint32_t wc = (uint32_t)__builtin_ctzll(__ballot(lane < kRW && g_start < l_start && g_start + wg >= l_start - wl));
            const uint32_t cs0 = wc * spw, csn = cs0 >= ns ? 0u : (ns - cs0 < spw ? ns - cs0 : spw);
            uint32_t gcar = lane_read(g_start, (int)wc), lcar = lane_read(l_start, (int)wc), sc = kNone;
            for (uint32_t j0 = 0; j0 < csn && sc == kNone; j0 += 64) {
                const uint32_t j = j0 + (uint32_t)lane;
                const uint64_t a = j < csn ? mge[cs0 + j] : 0ull, bb = j < csn ? mle[cs0 + j] : 0ull;
                const uint32_t cg = (uint32_t)__popcll(a), cl = (uint32_t)__popcll(bb);
                const uint32_t gi = wave_incl_scan(cg), li = wave_incl_scan(cl);
                const uint32_t gs = gcar + gi - cg, ls = lcar - (li - cl);
                const uint64_t hit = __ballot(j < csn && gs < ls && gs + cg >= ls - cl);
                if (hit) {
                    const int L = __builtin_ctzll(hit);
                    sc = cs0 + j0 + (uint32_t)L;
                    gcar = lane_read(gs, L);
                    lcar = lane_read(ls, L);
                } else {
                    gcar += lane_read(gi, 63);
                    lcar -= lane_read(li, 63);
                }
            }
            const uint64_t a = mge[sc], bb = mle[sc];
            uint32_t lo = 1, hi = 64;  // smallest b with G(b) >= Lc(b) inside step sc
            while (lo < hi) {
                const uint32_t m = (lo + hi) / 2;
                const uint64_t lm = low_mask(m);
                if (gcar + (uint32_t)__popcll(a & lm) >= lcar - (uint32_t)__popcll(bb & lm)) hi = m;
                else lo = m + 1;
            }
            const uint32_t g1 = gcar + (uint32_t)__popcll(a & low_mask(lo - 1));
            const uint32_t l2 = lcar - (uint32_t)__popcll(bb & low_mask(lo));
            ks = uni(g1 > l2 ? g1 : l2);
        }
        phase(2);
        // ---- the swap partners of the wave's steps
        // the lists: LDS segments keep them beside the segment; with 16-bit positions, a segment in global
        // memory keeps them in the (then idle) LDS segment area, 32768 entries each (Ks <= S / 2 <= 32768)
        const bool big = sizeof(Id) == 2 && where != kLds;
        uint16_t* const lpl = big ? reinterpret_cast<uint16_t*>(sh.key) : sh.lp;
        uint16_t* const rpl = big ? reinterpret_cast<uint16_t*>(sh.key) + 32768 : sh.rp;
        const bool lds_lists = where == kLds || big;
        uint32_t gpr[R], lsr[R];
#pragma unroll
        for (int r = 0; r < R; ++r) { gpr[r] = gb + gex[r]; lsr[r] = lt - lb - lex[r]; }
        partners<R>(b0, ws0, wsn, ks, mg, ml, gpr, lsr, lds_lists, lpl, rpl);
        __syncthreads();
        phase(3);
        const uint32_t cut_l = uni(sh.cut_l), cut_r = ks > 0 ? uni(sh.cut_r) : kNone;
        const uint32_t cut = cut_l < cut_r ? cut_l : cut_r;
        const bool right = cut <= nth;  // the side introselect continues with
        const uint32_t nf = right ? cut : first, nl = right ? last : cut;
        auto lpos = [&](uint32_t k) { return lds_lists ? b0 + lpl[k] : glp[k]; };  // L_{k+1}
        auto rpos = [&](uint32_t k) { return lds_lists ? b0 + rpl[k] : grp[k]; };  // R_{k+1}
        // ---- vec[nth - 1] after this partition, if this cut leaves it behind for good
        if (cut == nth && !rec) {
            lo_el = (ks > 0 && sh.l_ks == cut - 1) ? elp(cut_r) : elp(cut - 1);
            __syncthreads();  // read before any swap (block-uniform branch)
        }
        if (where == kSrc) {
            // ---- copy the surviving side out of the read-only keys (coalesced), then the swap targets take
            // their partners
            uint32_t nb = nf & ~63u;
            // (16-bit positions: the lists occupy the LDS segment area, so the survivors go to global memory
            // and move to LDS at the next round)
            const int dst = !big && (nl - nb) <= (uint32_t)kCap && M <= (sizeof(Id) == 2 ? 65536u : 0xFFFFFFFFu) ? kLds : kGlb;
            if (dst == kGlb) nb = 0;
            const uint32_t n = nl - nf;
            for (uint32_t i0 = (uint32_t)tid; i0 < n; i0 += kRT * 8) {
                uint32_t kk[8];
#pragma unroll
                for (int b = 0; b < 8; ++b) {
                    const uint32_t i = i0 + (uint32_t)(kRT * b);
                    kk[b] = i < n ? Src::key_at(kb, nf + i) : 0u;
                }
#pragma unroll
                for (int b = 0; b < 8; ++b) {
                    const uint32_t i = i0 + (uint32_t)(kRT * b), p = nf + i;
                    if (i >= n) break;
                    const El e = p == first ? pv.e : (p == pv.ch ? pv.f0 : El{kk[b], p});
                    if (dst == kLds) { sh.key[p - nb] = e.key; sh.id[p - nb] = (Id)e.id; }
                    else { gkey[p] = e.key; gid[p] = e.id; }
                }
            }
            __syncthreads();
            for (uint32_t k0 = (uint32_t)tid; k0 < ks; k0 += kRT * kBatch) {
                uint32_t to[kBatch];
                El ev[kBatch];
#pragma unroll
                for (int b = 0; b < kBatch; ++b) {
                    const uint32_t k = k0 + (uint32_t)(kRT * b);
                    if (k < ks) {
                        const uint32_t lq = lpos(k), rq = rpos(k);
                        to[b] = right ? rq : lq;
                        ev[b] = elp(right ? lq : rq);
                    }
                }
#pragma unroll
                for (int b = 0; b < kBatch; ++b) {
                    if (k0 + (uint32_t)(kRT * b) >= ks) break;
                    if (dst == kLds) { sh.key[to[b] - nb] = ev[b].key; sh.id[to[b] - nb] = (Id)ev[b].id; }
                    else { gkey[to[b]] = ev[b].key; gid[to[b]] = ev[b].id; }
                }
            }
            where = dst;
            base = nb;
        } else {
            // ---- in place, on the surviving side only: R_k <- old L_k (right) or L_k <- old R_k (left).
            // Reads (one side) and writes (the other) are disjoint; the two positions of the median-of-three
            // swap are read from pv (registers) and written by thread 0 unless a swap target
            for (uint32_t k0 = (uint32_t)tid; k0 < ks; k0 += kRT * kBatch) {
                uint32_t to[kBatch];
                El ev[kBatch];
#pragma unroll
                for (int b = 0; b < kBatch; ++b) {
                    const uint32_t k = k0 + (uint32_t)(kRT * b);
                    if (k < ks) {
                        const uint32_t lq = lpos(k), rq = rpos(k);
                        to[b] = right ? rq : lq;
                        ev[b] = elp(right ? lq : rq);
                    }
                }
#pragma unroll
                for (int b = 0; b < kBatch; ++b)
                    if (k0 + (uint32_t)(kRT * b) < ks) put(to[b], ev[b]);
            }
            if (tid == 0) {
                if (first >= nf && first < nl) put(first, pv.e);
                if (pv.ch >= nf && pv.ch < nl) {  // is ch a swap target? its ranks from the step records
                    const uint32_t s = (pv.ch - b0) / 64, bit = (pv.ch - b0) % 64;
                    const uint64_t below = low_mask(bit), a = mge[s], bb = mle[s];
                    const uint32_t g0 = mgp[s], l0 = mls[s];
                    bool tgt = false;
                    if (!right && ((a >> bit) & 1ull)) tgt = g0 + (uint32_t)__popcll(a & below) + 1 <= ks;
                    if (right && ((bb >> bit) & 1ull)) tgt = l0 - (uint32_t)__popcll(bb & below) <= ks;
                    if (!tgt) put(pv.ch, pv.f0);
                }
            }
        }
        __syncthreads();
        phase(4);
        rec = rec || cut == nth;
        first = nf;
        last = nl;
    }

    // ---------------------------------------------------------------- one round of a small LDS segment
    // (<= 64 steps) by one wave, no barriers: lane = step for the records, lane = bit for the partners.
    // LDS accesses of one wave complete in program order, so a lane reads what another lane wrote in an
    // earlier instruction.
    __device__ __forceinline__ void wave_round() {
        first = uni(first); last = uni(last);
        const uint32_t b0 = first & ~63u, ns = (last - b0 + 63) / 64;
        uint64_t tp = kSt ? clock64() : 0;
        const uint64_t t_start = tp;
        uint32_t t_sweep = 0;
        auto phase = [&](int i) {  // diagnostics: cycles per phase of the wave rounds
            if (kSt && lane == 0) {
                const uint64_t t = clock64();
                sh.stamp[23 + i] += t - tp;
                if (i == 1) t_sweep = (uint32_t)(t - tp);
                if (i == 4 && sh.nwlog < 22) {
                    sh.wlog[sh.nwlog][0] = ns; sh.wlog[sh.nwlog][1] = t_sweep; sh.wlog[sh.nwlog][2] = (uint32_t)(t - t_start);
                    sh.nwlog = sh.nwlog + 1;
                }
                tp = t;
            }
        };
        choose_pivot();
        pv = uni(pv);
        if (lane == 0) { sh.cut_l = kNone; sh.cut_r = kNone; sh.l_ks = kNone; }
        const uint32_t f0c = classify(pv.f0.key, pv.ch);
        uint64_t mg[R], ml[R];  // row 0 only (ns <= 64): the block round's instantiations, no extra code
        phase(0);
        sweep_rows<R>(b0, 0, ns, mg, ml);
        fix_rows<R>(b0, 0, ns, f0c, mg, ml);
        phase(1);
        const uint32_t cg = (uint32_t)__popcll(mg[0]), cl = (uint32_t)__popcll(ml[0]);
        const uint32_t gi = wave_incl_scan(cg), li = wave_incl_scan(cl);
        const uint32_t lt = lane_read(li, 63);
        const uint32_t gpre = gi - cg, lsuf = lt - (li - cl);
        // ---- crossing
        const uint64_t hit = __ballot((uint32_t)lane < ns && gpre < lsuf && gpre + cg >= lsuf - cl);
        const int sc = __builtin_ctzll(hit);
        const uint64_t a = lane_read_u64(mg[0], sc), bb = lane_read_u64(ml[0], sc);
        const uint32_t gcar = lane_read(gpre, sc), lcar = lane_read(lsuf, sc);
        uint32_t lo = 1, hi = 64;
        while (lo < hi) {
            const uint32_t m = (lo + hi) / 2;
            const uint64_t lm = low_mask(m);
            if (gcar + (uint32_t)__popcll(a & lm) >= lcar - (uint32_t)__popcll(bb & lm)) hi = m;
            else lo = m + 1;
        }
        const uint32_t g1 = gcar + (uint32_t)__popcll(a & low_mask(lo - 1));
        const uint32_t l2 = lcar - (uint32_t)__popcll(bb & low_mask(lo));
        const uint32_t ks = g1 > l2 ? g1 : l2;
        // ---- partners (lists in LDS) and L_{Ks+1}, L_{Ks}, R_{Ks}
        {
            uint32_t gpr[R], lsr[R];
#pragma unroll
            for (int r = 0; r < R; ++r) { gpr[r] = gpre; lsr[r] = lsuf; }
            phase(2);
            partners<R>(b0, 0, ns, ks, mg, ml, gpr, lsr, true, sh.lp, sh.rp);
        }
        const uint32_t cut_l = __builtin_amdgcn_readfirstlane(sh.cut_l);
        phase(3);
        const uint32_t cut_r = __builtin_amdgcn_readfirstlane(sh.cut_r);
        const uint32_t l_ks = __builtin_amdgcn_readfirstlane(sh.l_ks);
        const uint32_t cut = cut_l < cut_r ? cut_l : cut_r;
        const bool right = cut <= nth;
        const uint32_t nf = right ? cut : first, nl = right ? last : cut;
        if (cut == nth && !rec) lo_el = (ks > 0 && l_ks == cut - 1) ? elp(cut_r) : elp(cut - 1);
        // ---- swaps, then the median-of-three swap (lane 0; ch's target test from its step's records)
        const uint32_t s = (pv.ch - b0) / 64, bit = (pv.ch - b0) % 64;
        const uint64_t ga = lane_read_u64(mg[0], (int)s), la = lane_read_u64(ml[0], (int)s), below = low_mask(bit);
        const uint32_t g0 = lane_read(gpre, (int)s), l0 = lane_read(lsuf, (int)s);
        bool tgt = false;
        if (!right && ((ga >> bit) & 1ull)) tgt = g0 + (uint32_t)__popcll(ga & below) + 1 <= ks;
        if (right && ((la >> bit) & 1ull)) tgt = l0 - (uint32_t)__popcll(la & below) <= ks;
        for (uint32_t k0 = (uint32_t)lane; k0 < ks; k0 += 64 * kBatch) {
            uint32_t to[kBatch];
            El ev[kBatch];
#pragma unroll
            for (int b = 0; b < kBatch; ++b) {
                const uint32_t k = k0 + (uint32_t)(64 * b);
                if (k < ks) {
                    const uint32_t lq = b0 + sh.lp[k], rq = b0 + sh.rp[k];
                    to[b] = right ? rq : lq;
                    ev[b] = elp(right ? lq : rq);
                }
            }
#pragma unroll
            for (int b = 0; b < kBatch; ++b)
                if (k0 + (uint32_t)(64 * b) < ks) put(to[b], ev[b]);
        }
        if (lane == 0) {
            if (first >= nf && first < nl) put(first, pv.e);
            if (pv.ch >= nf && pv.ch < nl && !tgt) put(pv.ch, pv.f0);
        }
        __builtin_amdgcn_wave_barrier();
        phase(4);
        rec = rec || cut == nth;
        first = nf;
        last = nl;
    }

    // ---------------------------------------------------------------- rounds of a segment of <= 64 elements
    // One wave, lane = position - first, the elements in registers: the median of three by readlane, the
    // masks by compares (as step_masks, restricted to the segment), Ks = max_t min(G(t), Lc(t)) by a wave max,
    // each swap partner by a bit select on the masks, the swaps by ds_bpermute; vec[nth - 1] recorded from
    // registers; the segment goes back to LDS once at the end.  Stops at <= 3 elements or depth 0.
    __device__ __forceinline__ void lane_rounds(uint32_t& nrounds) {
        first = uni(first); last = uni(last);
        const uint32_t S0 = last - first, base0 = first;
        const uint32_t me = (uint32_t)lane;
        El e = me < S0 ? get(base0 + me) : El{kKeyInvisible, 0u};
        uint32_t f = 0, l = S0;  // the segment, relative to base0
        const uint32_t nrel = nth - base0;
        const uint64_t below = low_mask(me);
        while (l - f > 3 && depth > 0) {
            --depth;
            ++nrounds;
            const uint32_t A = f + 1, B = f + (l - f) / 2, C = l - 1;
            const El a{lane_read(e.key, (int)A), lane_read(e.id, (int)A)};
            const El b{lane_read(e.key, (int)B), lane_read(e.id, (int)B)};
            const El c{lane_read(e.key, (int)C), lane_read(e.id, (int)C)};
            uint32_t ch;
            El pe;
            if (less(src, P, med, a, b)) {
                if (less(src, P, med, b, c)) { ch = B; pe = b; }
                else if (less(src, P, med, a, c)) { ch = C; pe = c; }
                else { ch = A; pe = a; }
            } else if (less(src, P, med, a, c)) { ch = A; pe = a; }
            else if (less(src, P, med, b, c)) { ch = C; pe = c; }
            else { ch = B; pe = b; }
            const El f0{lane_read(e.key, (int)f), lane_read(e.id, (int)f)};
            pivot_fields(uni(pe));
            pv = uni(pv);
            // the median-of-three swap (first <-> ch), then the masks over the segment
            if (me == f) e = pv.e;
            else if (me == ch) e = f0;
            const Thr t = thresholds();
            uint64_t ge, le, sl;
            if (P == 0) step_masks<0>(t, e.key, ge, le, sl);
            else step_masks<1>(t, e.key, ge, le, sl);
            const uint64_t in_ge = low_mask(l) & ~low_mask(f + 1), in_le = low_mask(l) & ~low_mask(f);
            sl &= in_ge;
            if (sl) {
                const bool mine = (sl >> me) & 1ull;
                uint32_t cc = 0;
                if (mine) cc = classify_slow(src, P, med, e.key, e.id, pv.e, pv.plo, pv.phi, kSt ? &sh.stamp[28 + P] : nullptr);
                ge = (ge & ~sl) | __ballot(mine && (cc & 1u));
                le = (le & ~sl) | __ballot(mine && (cc & 2u));
            }
            ge &= in_ge;
            le = (le & in_le) | (1ull << f);
            // Ks: split t in [f+1, l) (t = l adds min(G, 0) = 0)
            const uint32_t G = (uint32_t)__popcll(ge & below), Lc = (uint32_t)__popcll(le & ~below);
            const uint32_t mm = (me >= f + 1 && me < l) ? (G < Lc ? G : Lc) : 0u;
            const uint32_t ks = wave_max_u(mm);
            // ranks: L_k = k-th GE from the left, R_k = k-th LE from the right
            const bool isg = (ge >> me) & 1ull, isl = (le >> me) & 1ull;
            const uint32_t kg = G + 1u, kl = Lc;  // this lane's GE rank / LE right-rank (when set)
            const uint32_t cg = (uint32_t)__popcll(ge);
            // L_{Ks+1} and R_{Ks} (kNone when absent), L_{Ks}
            const uint32_t cut_l = ks + 1u <= cg ? wave_min_u(isg && kg == ks + 1u ? me : kNone) : kNone;
            const uint32_t cut_r = ks > 0 ? wave_min_u(isl && kl == ks ? me : kNone) : kNone;
            const uint32_t cut = cut_l < cut_r ? cut_l : cut_r;
            // swap partners: the L_k lane takes R_k, the R_k lane takes L_k (k <= Ks)
            uint32_t src_lane = me;
            if (isg && kg <= ks) src_lane = 63u - select_bit(__builtin_bitreverse64(le), kg - 1u);
            if (isl && kl <= ks) src_lane = select_bit(ge, kl - 1u);
            const El ne{(uint32_t)__builtin_amdgcn_ds_bpermute((int)(src_lane * 4u), (int)e.key),
                        (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src_lane * 4u), (int)e.id)};
            e = ne;
            const bool right = cut <= nrel;
            if (cut == nrel && !rec && nrel >= 1) lo_el = El{lane_read(e.key, (int)(cut - 1)), lane_read(e.id, (int)(cut - 1))};
            rec = rec || cut == nrel;
            if (right) f = cut;
            else l = cut;
        }
        if (me < S0) put(base0 + me, e);
        __builtin_amdgcn_wave_barrier();
        first = base0 + f;
        last = base0 + l;
    }

    // ---------------------------------------------------------------- std::nth_element(vec, vec + nth)
    // (vec[nth - 1], vec[nth]) of the post-state as values (lo only when nth >= 1), on thread 0
    __device__ __forceinline__ void select(double& lo, double& hi) {
        first = 0; last = M; base = 0; where = kSrc; rec = 0;
        depth = M > 1 ? 2 * lg2(M) : 0;
        const uint64_t t0 = kSt ? clock64() : 0;
        uint64_t t1 = t0;
        uint32_t nblk = 0, nwave = 0;
        while (last - first > 3) {
            if (depth == 0) {
                if (tid == 0)
                    heap_select_fn<Src, Id>(HeapView<Src, Id>{src, &sh, gkey, gid, first, base, where, P, med},
                                            nth + 1 - first, last - first, nth - first);
                __syncthreads();
                break;
            }
            if (where == kLds && last - (first & ~63u) <= 64u * kWaveSteps) {  // the rest by wave 0, no barriers
                if (wave == 0) {
                    while (last - first > 3 && depth > 0) {
                        if (last - first <= 64u) {
                            lane_rounds(nwave);
                            break;
                        }
                        --depth;
                        wave_round();
                        ++nwave;
                    }
                    if (lane == 0) {
                        sh.bc_first = first; sh.bc_last = last; sh.bc_depth = (uint32_t)depth; sh.bc_rec = (uint32_t)rec;
                        sh.lo_el = lo_el;
                    }
                }
                __syncthreads();
                first = uni(sh.bc_first); last = uni(sh.bc_last); depth = (int)uni(sh.bc_depth); rec = (int)uni(sh.bc_rec);
                lo_el = uni(sh.lo_el);
                __syncthreads();
                continue;  // depth 0 with > 3 left: the heap select above
            }
            --depth;
            if (where == kGlb && last - (first & ~63u) <= (uint32_t)kCap && M <= (sizeof(Id) == 2 ? 65536u : 0xFFFFFFFFu)) {
                const uint32_t nb = first & ~63u;  // the segment now fits in LDS
                for (uint32_t p = first + tid; p < last; p += kRT) {
                    sh.key[p - nb] = gkey[p];
                    sh.id[p - nb] = (Id)gid[p];
                }
                where = kLds;
                base = nb;
                __syncthreads();
            }
            {
                const uint64_t tb = kSt ? clock64() : 0;
                const uint32_t S = last - first, w = (uint32_t)where;
                round();
                if (kSt && tid == 0 && sh.nblog < 40) {
                    sh.blog[sh.nblog][0] = S; sh.blog[sh.nblog][1] = w; sh.blog[sh.nblog][2] = (uint32_t)(clock64() - tb);
                    sh.nblog = sh.nblog + 1;
                }
            }
            ++nblk;
            if (kSt && nblk == 1) t1 = clock64();
        }
        if (kSt && tid == 0) {
            sh.stamp[4 * P] = t1 - t0;
            sh.stamp[4 * P + 1] = clock64() - t1;
            sh.stamp[4 * P + 2] = nblk;
            sh.stamp[4 * P + 3] = nwave;
        }
        if (tid == 0) {
            if (last - first <= 3) {  // std::__insertion_sort of the last <= 3
                const uint32_t n = last - first;
                El v[3];
                for (uint32_t i = 0; i < n; ++i) v[i] = get(first + i);
                for (uint32_t i = 1; i < n; ++i) {
                    const El x = v[i];
                    uint32_t j = i;
                    while (j > 0 && less(src, P, med, x, v[j - 1])) { v[j] = v[j - 1]; --j; }
                    v[j] = x;
                }
                for (uint32_t i = 0; i < n; ++i) sh.fin[i] = v[i];
                hi = value(src, P, med, sh.fin[nth - first]);
                if (nth >= 1) lo = value(src, P, med, rec ? lo_el : sh.fin[nth - 1 - first]);
            } else {  // heap select ran
                hi = value(src, P, med, get(nth));
                if (nth >= 1) lo = value(src, P, med, rec ? lo_el : get(nth - 1));
            }
        }
    }
};

// computeMedian / computeMAD (src/algorithm.cpp:834-865) with the reference's post-state: thread 0 of the
// block gets med and mad.  M slots, n visible.
template <typename Id, bool kSt, class Src>
__device__ __forceinline__ void ref_robust_scale(const Src& src, RefShared<Id>& sh, uint32_t* sel, int64_t sel_stride,
                                                 uint32_t M, uint32_t n, double& med, double& mad) {
    const int tid = (int)threadIdx.x;
    __shared__ Src src_sh;
    if (tid == 0) src_sh = src;
    __syncthreads();
    RefSel<Src, Id, kSt> s{&src_sh, sh};
    s.kb = src.kbase();
    const int64_t q = sel_stride / 4;  // q >= M entries each: keys, ids, step records, partner lists
    s.gkey = sel;
    s.gid = sel + q;
    const int64_t steps = (q + 63) / 64 + 1;
    s.gmge = reinterpret_cast<uint64_t*>(sel + 2 * q);
    s.gmle = s.gmge + steps;
    s.ggpre = reinterpret_cast<uint32_t*>(s.gmle + steps);
    s.glsuf = s.ggpre + steps;
    s.glp = sel + 3 * q;
    s.grp = sel + 3 * q + q / 2;
    s.M = M;
    s.nth = n / 2;
    s.tid = tid; s.lane = tid & 63; s.wave = uni(tid >> 6);
    s.med = 0.0;
    const bool even = (M & 1u) == 0 && s.nth >= 1;  // mid == 0 (UB in the reference) reads vec[mid]
    __shared__ double bc;
    for (int P = 0; P < 2; ++P) {  // one copy of the selection for both passes
        s.P = P;
        double lo = 0.0, hi = 0.0;
        s.select(lo, hi);
        if (tid == 0) {
            const double v = even ? (lo + hi) / 2.0 : hi;
            if (P == 0) { bc = v; med = v; }
            else mad = v;
        }
        __syncthreads();
        s.med = uni(bc);
    }
}

template <typename Id>
__device__ __forceinline__ void scale_ref_pair(const AlignArgs& a, int level, RefShared<Id>& sh) {
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
    if (lane == 0) { sh.wsum[wave][0] = nrv; sh.wsum[wave][1] = ncv; }
    __syncthreads();
    nrv = 0; ncv = 0;
    for (int w = 0; w < kRW; ++w) { nrv += sh.wsum[w][0]; ncv += sh.wsum[w][1]; }
    __syncthreads();
    const uint32_t n = ncv * (uint32_t)a.area;
    double med = kDblMax, mad = 0.0;  // n == 0: every slot is DBL_MAX in the reference
    if (n > 0) {
        ImgSrc src;
        src.keys = a.keys32 + (int64_t)pair * a.key_stride;
        src.px = a.px + (int64_t)pair * a.max_f * 2;
        src.cproj = a.cproj + (int64_t)pair * a.max_f * 2;
        src.rplane = P.ref_pyr + a.geom.off[level];
        src.kplane = P.kf_pyr + a.geom.off[level];
        src.cplane = P.cur_pyr + a.geom.off[level];
        src.W = a.geom.w[level];
        src.area = a.area;
        src.side = 2 * a.half + 1;
        src.half = a.half;
        src.n_ref = P.n_ref;
        src.scale = ldexp(1.0, -level);
        ref_robust_scale<Id, false>(src, sh, a.sel + (int64_t)pair * a.sel_stride, a.sel_stride, M, n, med, mad);
    }
    if (tid == 0) {
        double sigma = 1.482602218505602 * mad;
        if (sigma <= 2.220446049250313e-16) sigma = 2.220446049250313e-16;
        S.med = med;
        S.mad = mad;
        S.sigma = sigma;
        S.c = 4.6851 * sigma;
        S.n = n;
        S.n_ref_vis = nrv;
    }
}

}  // namespace

// K2R: one workgroup per pair (replaces align_scale_kernel when median_mode = SVO_MEDIAN_REFERENCE).
// Id: 16-bit slot ids in LDS when every pair's vector has <= 65536 slots, else 32-bit.
template <typename Id>
__global__ void __launch_bounds__(kRT, 1) align_scale_ref_kernel(AlignArgs a, int level) {
    __shared__ RefShared<Id> sh;
    scale_ref_pair<Id>(a, level, sh);
}

// svo_debug_robust_scale: the same selection on an arbitrary residual vector (one workgroup)
template <typename Id>
__global__ void __launch_bounds__(kRT, 1) debug_robust_scale_kernel(const double* v, uint32_t M, uint32_t n,
                                                                   uint32_t* sel, int64_t sel_stride, double* out,
                                                                   int flags) {
    __shared__ RefShared<Id> sh;
    if (threadIdx.x < 32) sh.stamp[threadIdx.x] = 0;
    if (threadIdx.x == 0) { sh.nwlog = 0; sh.nblog = 0; }
    (void)flags;
    // the keys K1 would have written (res_key32), into the tail of the scratch
    const int64_t q = sel_stride / 4;
    uint32_t* keys = sel + 4 * q;  // (svo_debug_robust_scale allocates 5 q)
    for (uint32_t p = threadIdx.x; p < M; p += kRT) keys[p] = v[p] >= kDblMax ? kKeyInvisible : res_key32(v[p]);
    __threadfence_block();
    __syncthreads();
    ArrSrc src{v, keys};
    double med = 0.0, mad = 0.0;
    ref_robust_scale<Id, true>(src, sh, sel, sel_stride, M, n, med, mad);
    if (threadIdx.x == 0) {
        out[0] = med;
        out[1] = mad;
        for (int i = 0; i < 30; ++i) out[2 + i] = (double)sh.stamp[i];
        for (int i = 0; i < 66; ++i) out[32 + i] = i / 3 < (int)sh.nwlog ? (double)sh.wlog[i / 3][i % 3] : -1.0;
        for (int i = 0; i < 120; ++i) out[98 + i] = i / 3 < (int)sh.nblog ? (double)sh.blog[i / 3][i % 3] : -1.0;
    }
}

int ref_threads() { return kRT; }
void launch_scale_ref(const AlignArgs& a, int level, hipStream_t s) {
    if ((int64_t)a.max_f * a.area <= 65536)
        hipLaunchKernelGGL(align_scale_ref_kernel<uint16_t>, dim3(a.n_pairs), dim3(kRT), 0, s, a, level);
    else
        hipLaunchKernelGGL(align_scale_ref_kernel<uint32_t>, dim3(a.n_pairs), dim3(kRT), 0, s, a, level);
}
void launch_debug_robust_scale(const double* v, uint32_t M, uint32_t n, uint32_t* sel, int64_t sel_stride, double* out,
                               int flags, hipStream_t s) {
    if (M <= 65536)
        hipLaunchKernelGGL(debug_robust_scale_kernel<uint16_t>, dim3(1), dim3(kRT), 0, s, v, M, n, sel, sel_stride, out, flags);
    else
        hipLaunchKernelGGL(debug_robust_scale_kernel<uint32_t>, dim3(1), dim3(kRT), 0, s, v, M, n, sel, sel_stride, out, flags);
}

}  // namespace svo
