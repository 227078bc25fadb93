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
// does.  A round classifies every element once, keeping per-64-position-step GE / LE ballots; the scans,
// the crossing, L_{Ks+1} / R_{Ks} and each swap's partners come from those records (four barriers).
#include "svo_internal.h"
#include "svo_math.h"
#include "svo_wave.h"

namespace svo {

namespace {

constexpr int kRT = 1024;              // threads per pair
constexpr int kRW = kRT / 64;          // waves
constexpr int kMeta = 1024;            // LDS step records (64 positions each): segments up to 65536
constexpr int kBatch = 4;              // sweeps: 256-position groups whose loads a wave issues before using any
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
};

template <typename Id>
struct RefShared {
    static constexpr int kCap = sizeof(Id) == 2 ? 16384 : 12288;  // LDS segment capacity (elements)
    alignas(16) uint32_t key[kCap];          // the segment, from position `base`
    Id id[kCap];
    uint16_t lp[kCap / 2], rp[kCap / 2];     // L_k, R_k - b0 for k <= Ks (LDS rounds)
    uint64_t mge[kMeta], mle[kMeta];         // per 64-position step: GE / LE ballots
    uint32_t gpre[kMeta], lsuf[kMeta];       // GE before the step; LE from the step's start on
    uint32_t wsum[kRW][2];
    uint32_t ks, cut_l, cut_r, l_ks;
    El fin[3];
    uint64_t stamp[32];  // diagnostics (svo_debug_robust_scale): per pass: cycles of round 1, of the rest, rounds;
                         // then cycles per (round kind, phase) summed over both passes
};

// where the current segment lives
enum { kSrc = 0, kGlb = 1, kLds = 2 };

// ---- element sources: round-1 keys in the reference's order, and the exact residual of a slot
struct ImgSrc {  // production: K1's keys and the images
    const uint32_t* keys;   // pair's feature-major keys: slot f * area + k (padded: 16-B reads past M are safe)
    const double* px;       // pair's feature pixels (level 0)
    const double* cproj;    // pair's projections into the cur level (K1)
    const uint8_t *rplane, *kplane, *cplane;
    int W, area, side, half, n_ref;
    double scale;
    __device__ __forceinline__ uint32_t key(uint32_t p) const { return keys[p]; }
    __device__ __forceinline__ uint4 key4(uint32_t p) const { return *reinterpret_cast<const uint4*>(keys + p); }
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
struct ArrSrc {  // svo_debug_robust_scale: an arbitrary residual vector (>= DBL_MAX = invisible), padded
    const double* v;
    __device__ __forceinline__ uint32_t key(uint32_t p) const { return v[p] >= kDblMax ? kKeyInvisible : res_key32(v[p]); }
    __device__ __forceinline__ uint4 key4(uint32_t p) const { return make_uint4(key(p), key(p + 1), key(p + 2), key(p + 3)); }
    __device__ __forceinline__ double r(uint32_t s) const { return v[s]; }
};

__device__ __forceinline__ int lg2(uint32_t n) { return 31 - __builtin_clz(n); }

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
// bits 0..15 of v to bits 0, 4, 8, .., 60
__device__ __forceinline__ uint64_t spread4(uint64_t v) {
    uint64_t x = v & 0xFFFFull;
    x = (x | (x << 24)) & 0x000000FF000000FFull;
    x = (x | (x << 12)) & 0x000F000F000F000Full;
    x = (x | (x << 6)) & 0x0303030303030303ull;
    x = (x | (x << 3)) & 0x1111111111111111ull;
    return x;
}
__device__ __forceinline__ uint64_t low_mask(uint32_t b) { return b >= 64 ? ~0ull : ((1ull << b) - 1ull); }

// the exact comparison of an element with the pivot (rare: equal key cells); a free function of values so
// that the selection state stays in registers
template <int P, class Src>
__device__ __attribute__((noinline)) uint32_t classify_exact(Src src, uint32_t ek, uint32_t eid, uint32_t pk, uint32_t pid,
                                                            double med) {
    auto val = [&](uint32_t k, uint32_t id) {
        if (k == kKeyInvisible) return kDblMax;
        const double r = (k & 1u) ? src.r(id) : key_r(k);
        return P == 0 ? r : fabs(r - med);
    };
    const double v = val(ek, eid), p = val(pk, pid);
    return (!(v < p) ? 1u : 0u) | (!(p < v) ? 2u : 0u);
}

template <class Src, typename Id>
struct RefSel {
    using Shared = RefShared<Id>;
    static constexpr int kCap = Shared::kCap;
    Src src;
    Shared& sh;
    uint32_t* gkey;   // pair's global segment keys / ids (absolute positions)
    uint32_t* gid;
    uint32_t* glp;    // swap partners L_k / R_k of the global and copy rounds
    uint32_t* grp;
    uint64_t* gmge;   // step records of segments past kMeta steps
    uint64_t* gmle;
    uint32_t* ggpre;
    uint32_t* glsuf;
    uint32_t M, nth;
    double med;       // pass 1
    int tid, lane, wave;
    // block-uniform state
    uint32_t first, last, base;
    int where, depth, rec;
    El lo_el;
    Pivot pv;

    // ---------------------------------------------------------------- values and comparisons
    template <int P>
    __device__ __forceinline__ double value(El e) const {  // the reference's vector entry (exact)
        if (e.key == kKeyInvisible) return kDblMax;
        const double r = (e.key & 1u) ? src.r(e.id) : key_r(e.key);
        return P == 0 ? r : fabs(r - med);
    }
    __device__ __forceinline__ void d_interval(uint32_t k, double& lo, double& hi) const {  // |r - med| over the key's cell
        const double rl = key_r(k), rh = (k & 1u) ? rl + kKeyStep : rl;
        if (rh <= med) { lo = med - rh; hi = med - rl; }
        else if (rl >= med) { lo = rl - med; hi = rh - med; }
        else { lo = 0.0; hi = fmax(med - rl, rh - med); }
    }
    template <int P>
    __device__ __forceinline__ bool less(El a, El b) const {  // value(a) < value(b)
        if (P == 0) {
            if (a.key != b.key) return a.key < b.key;
            if (a.key == kKeyInvisible || !(a.key & 1u)) return false;
            return value<0>(a) < value<0>(b);
        } else {
            if (a.key == kKeyInvisible) return false;
            if (b.key == kKeyInvisible) return true;
            double alo, ahi, blo, bhi;
            d_interval(a.key, alo, ahi);
            d_interval(b.key, blo, bhi);
            if (ahi < blo) return true;
            if (alo >= bhi) return false;
            return value<1>(a) < value<1>(b);
        }
    }
    // (ge, le) = (!(a < p), !(p < a)) as bits 0, 1 for the element of key k at position p
    template <int P, int W>
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
            double lo, hi;
            d_interval(k, lo, hi);
            if (hi < pv.plo) return 2u;
            if (lo > pv.phi) return 1u;
        }
        return classify_exact<P, Src>(src, k, elp<W>(p).id, pv.e.key, pv.e.id, med);
    }
    template <int P>
    __device__ __forceinline__ void pivot_info() {  // the pass-1 interval and thresholds of pv.e
        pv.inv = pv.e.key == kKeyInvisible;
        if (P == 1 && !pv.inv) {
            d_interval(pv.e.key, pv.plo, pv.phi);
            pv.kA = key_grid(med - pv.plo);
            pv.kB = key_grid(med + pv.plo);
            pv.kC = key_grid(med - pv.phi);
            pv.kD = key_grid(med + pv.phi);
        }
    }

    // ---------------------------------------------------------------- storage
    template <int W>
    __device__ __forceinline__ El get(uint32_t p) const {
        if (W == kSrc) return El{src.key(p), p};
        if (W == kGlb) return El{gkey[p], gid[p]};
        return El{sh.key[p - base], (uint32_t)sh.id[p - base]};
    }
    template <int W>
    __device__ __forceinline__ uint4 get4(uint32_t p) const {  // keys p .. p+3 (p a multiple of 4)
        if (W == kSrc) return src.key4(p);
        if (W == kGlb) return *reinterpret_cast<const uint4*>(gkey + p);
        return *reinterpret_cast<const uint4*>(&sh.key[p - base]);
    }
    template <int W>
    __device__ __forceinline__ void put(uint32_t p, El e) {
        if (W == kGlb) { gkey[p] = e.key; gid[p] = e.id; }
        if (W == kLds) { sh.key[p - base] = e.key; sh.id[p - base] = (Id)e.id; }
    }
    // the segment after the median-of-three swap (first <-> ch), before it is stored
    template <int W>
    __device__ __forceinline__ El elp(uint32_t p) const {
        if (p == first) return pv.e;
        if (p == pv.ch) return pv.f0;
        return get<W>(p);
    }
    __device__ __forceinline__ El get_any(uint32_t p) const {
        if (where == kGlb) return get<kGlb>(p);
        if (where == kLds) return get<kLds>(p);
        return get<kSrc>(p);
    }
    __device__ __forceinline__ void put_any(uint32_t p, El e) {
        if (where == kGlb) put<kGlb>(p, e);
        else if (where == kLds) put<kLds>(p, e);
    }

    // ---------------------------------------------------------------- one partition round
    // Steps are 64 positions from b0 = first & ~63.  The classification sweep stores each step's GE / LE
    // ballots (16-B loads: a wave covers 256 positions, the four 64-lane ballots interleave into four
    // step records); the scans, the crossing, L_{Ks+1} / R_{Ks} and the swaps work from those records.
    // kLM: the step records live in LDS (segments up to kMeta steps) or in the global scratch.
    template <int P, int W, bool kLM>
    __device__ __forceinline__ void round() {
        const uint32_t S = last - first, b0 = first & ~63u, ns = (last - b0 + 63) / 64, ng = (ns + 3) / 4;
        uint64_t* const mge = kLM ? sh.mge : gmge;
        uint64_t* const mle = kLM ? sh.mle : gmle;
        uint32_t* const gpre = kLM ? sh.gpre : ggpre;
        uint32_t* const lsuf = kLM ? sh.lsuf : glsuf;
        uint64_t tp = clock64();
        auto phase = [&](int i) {
            if (tid == 0) { const uint64_t t = clock64(); sh.stamp[8 + 6 * W + i] += t - tp; tp = t; }
        };
        // ---- pivot: std::__move_median_to_first(first, first + 1, first + S/2, last - 1), computed by
        // every thread (same reads, same answer; no broadcast)
        {
            const uint32_t A = first + 1, B = first + S / 2, C = last - 1;
            const El a = get<W>(A), b = get<W>(B), c = get<W>(C);
            uint32_t ch;
            El e;
            if (less<P>(a, b)) {
                if (less<P>(b, c)) { ch = B; e = b; }
                else if (less<P>(a, c)) { ch = C; e = c; }
                else { ch = A; e = a; }
            } else if (less<P>(a, c)) { ch = A; e = a; }
            else if (less<P>(b, c)) { ch = C; e = c; }
            else { ch = B; e = b; }
            pv.e = e;
            pv.f0 = get<W>(first);
            pv.ch = ch;
            pivot_info<P>();
        }
        phase(0);
        // ---- classification sweep
        for (uint32_t g0 = (uint32_t)wave; g0 < ng; g0 += kRW * kBatch) {
            uint4 kv[kBatch];
#pragma unroll
            for (int b = 0; b < kBatch; ++b) {
                const uint32_t g = g0 + (uint32_t)(kRW * b), p = b0 + 256 * g + 4 * (uint32_t)lane;
                kv[b] = (g < ng && p < last) ? get4<W>(p) : make_uint4(0, 0, 0, 0);
            }
#pragma unroll
            for (int b = 0; b < kBatch; ++b) {
                const uint32_t g = g0 + (uint32_t)(kRW * b), p = b0 + 256 * g + 4 * (uint32_t)lane;
                if (g >= ng) break;  // wave-uniform
                const uint32_t kk[4] = {kv[b].x, kv[b].y, kv[b].z, kv[b].w};
                uint64_t bg[4], bl[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const uint32_t q = p + (uint32_t)j;
                    uint32_t c = 0;
                    if (q >= first && q < last) {
                        if (q == first) c = 2u;  // the pivot: the right scan's sentinel, outside the left scan
                        else c = classify<P, W>(q == pv.ch ? pv.f0.key : kk[j], q);
                    }
                    bg[j] = __ballot(c & 1u);
                    bl[j] = __ballot(c & 2u);
                }
                if (lane < 4) {  // lane q writes step 4 g + q: positions 64 q + 4 l + j hold lane 16 q + l, key j
                    const uint32_t s = 4 * g + (uint32_t)lane;
                    if (s < ns) {
                        uint64_t mg = 0, ml = 0;
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            mg |= spread4(bg[j] >> (16 * lane)) << j;
                            ml |= spread4(bl[j] >> (16 * lane)) << j;
                        }
                        mge[s] = mg;
                        mle[s] = ml;
                    }
                }
            }
        }
        __syncthreads();
        phase(1);
        // ---- scans over the steps: thread t owns steps [t * per, (t + 1) * per)
        const uint32_t per = (ns + kRT - 1) / kRT, s_lo = (uint32_t)tid * per;
        const uint32_t s_hi = s_lo + per < ns ? s_lo + per : ns;
        uint32_t gs = 0, ls = 0;
        for (uint32_t s = s_lo; s < s_hi; ++s) { gs += (uint32_t)__popcll(mge[s]); ls += (uint32_t)__popcll(mle[s]); }
        const uint32_t gi = wave_incl_scan(gs), li = wave_incl_scan(ls);
        if (lane == 63) { sh.wsum[wave][0] = gi; sh.wsum[wave][1] = li; }
        __syncthreads();
        phase(2);
        uint32_t gb = 0, lb = 0, lt = 0;
        for (int w = 0; w < kRW; ++w) {
            const uint32_t wg = sh.wsum[w][0], wl = sh.wsum[w][1];
            gb += w < wave ? wg : 0u;
            lb += w < wave ? wl : 0u;
            lt += wl;
        }
        // ---- per step G, Lc at its start; Ks = max_t min(G(t), Lc(t)): with t* the first split where
        // G >= Lc (G rises, Lc falls), Ks = max(G(t* - 1), Lc(t*)); the step holding t* finds it
        {
            uint32_t gex = gb + gi - gs, lfrom = lt - (lb + li - ls);
            for (uint32_t s = s_lo; s < s_hi; ++s) {
                const uint64_t mg = mge[s], ml = mle[s];
                gpre[s] = gex;
                lsuf[s] = lfrom;
                const uint32_t cg = (uint32_t)__popcll(mg), cl = (uint32_t)__popcll(ml);
                if (gex < lfrom && gex + cg >= lfrom - cl) {
                    uint32_t lo = 1, hi = 64;  // smallest b with G(b) >= Lc(b)
                    while (lo < hi) {
                        const uint32_t m = (lo + hi) / 2;
                        const uint64_t lm = low_mask(m);
                        if (gex + (uint32_t)__popcll(mg & lm) >= lfrom - (uint32_t)__popcll(ml & lm)) hi = m;
                        else lo = m + 1;
                    }
                    const uint32_t g1 = gex + (uint32_t)__popcll(mg & low_mask(lo - 1));
                    const uint32_t l2 = lfrom - (uint32_t)__popcll(ml & low_mask(lo));
                    sh.ks = g1 > l2 ? g1 : l2;
                }
                gex += cg;
                lfrom -= cl;
            }
        }
        if (tid == 0) { sh.cut_l = kNone; sh.cut_r = kNone; sh.l_ks = kNone; }
        __syncthreads();
        phase(3);
        const uint32_t ks = sh.ks;
        // ---- the swap partners: a wave takes a step, a lane a bit.  L_k (GE rank k <= Ks) and R_k (LE rank
        // k from the right) go to the lists lp / rp; L_{Ks+1}, L_{Ks} and R_{Ks} to shared scalars
        {
            uint16_t* const lp16 = sh.lp;
            uint16_t* const rp16 = sh.rp;
            for (uint32_t s = (uint32_t)wave; s < ns; s += kRW) {
                const uint64_t mg = mge[s], ml = mle[s];
                const uint32_t g0 = gpre[s], l0 = lsuf[s];
                const uint64_t below = low_mask((uint32_t)lane);
                const uint32_t pos = b0 + 64 * s + (uint32_t)lane;
                if (g0 < ks + 1 && ((mg >> lane) & 1ull)) {
                    const uint32_t k = g0 + (uint32_t)__popcll(mg & below) + 1;
                    if (k <= ks) {
                        if (W == kLds) lp16[k - 1] = (uint16_t)(pos - b0);
                        else glp[k - 1] = pos;
                    }
                    if (k == ks + 1) sh.cut_l = pos;
                    if (k == ks) sh.l_ks = pos;
                }
                if (l0 - (uint32_t)__popcll(ml) < ks && ((ml >> lane) & 1ull)) {
                    const uint32_t k = l0 - (uint32_t)__popcll(ml & below);
                    if (k <= ks) {
                        if (W == kLds) rp16[k - 1] = (uint16_t)(pos - b0);
                        else grp[k - 1] = pos;
                    }
                    if (k == ks) sh.cut_r = pos;
                }
            }
        }
        __syncthreads();
        phase(4);
        const uint32_t cut_l = sh.cut_l, cut_r = ks > 0 ? sh.cut_r : kNone;
        const uint32_t cut = cut_l < cut_r ? cut_l : cut_r;
        const bool right = cut <= nth;  // the side introselect continues with
        const uint32_t nf = right ? cut : first, nl = right ? last : cut;
        // ---- vec[nth - 1] after this partition, if this cut leaves it behind for good
        if (cut == nth && !rec) {
            lo_el = (ks > 0 && sh.l_ks == cut - 1) ? elp<W>(cut_r) : elp<W>(cut - 1);
            __syncthreads();  // read before any swap (block-uniform branch)
        }
        int dst = W;
        uint32_t nb = base;
        if (W == kSrc) {
            // ---- copy the surviving side out of the read-only keys (the swap targets follow)
            nb = nf & ~63u;
            dst = (nl - nb) <= (uint32_t)kCap && M <= (sizeof(Id) == 2 ? 65536u : 0xFFFFFFFFu) ? kLds : kGlb;
            if (dst == kGlb) nb = 0;
            const uint32_t n = nl - nf;
            for (uint32_t i0 = (uint32_t)tid; i0 < n; i0 += kRT * kBatch) {
                El ev[kBatch];
#pragma unroll
                for (int b = 0; b < kBatch; ++b) {
                    const uint32_t i = i0 + (uint32_t)(kRT * b);
                    if (i < n) ev[b] = elp<kSrc>(nf + i);
                }
#pragma unroll
                for (int b = 0; b < kBatch; ++b) {
                    const uint32_t i = i0 + (uint32_t)(kRT * b);
                    if (i < n) {
                        if (dst == kLds) { sh.key[nf + i - nb] = ev[b].key; sh.id[nf + i - nb] = (Id)ev[b].id; }
                        else { gkey[nf + i] = ev[b].key; gid[nf + i] = ev[b].id; }
                    }
                }
            }
            __syncthreads();
        }
        auto store = [&](uint32_t p, El e) {
            if (dst == kLds) { sh.key[p - nb] = e.key; sh.id[p - nb] = (Id)e.id; }
            else { gkey[p] = e.key; gid[p] = e.id; }
        };
        // ---- the swaps on the surviving side: R_k <- old L_k (right) or L_k <- old R_k (left), k <= Ks.
        // Reads (one side) and writes (the other) are disjoint; the two positions of the median-of-three
        // swap are read from pv (registers)
        for (uint32_t k0 = (uint32_t)tid; k0 < ks; k0 += kRT * kBatch) {
            uint32_t to[kBatch];
            El ev[kBatch];
#pragma unroll
            for (int b = 0; b < kBatch; ++b) {
                const uint32_t k = k0 + (uint32_t)(kRT * b);
                if (k < ks) {
                    const uint32_t lq = W == kLds ? b0 + sh.lp[k] : glp[k], rq = W == kLds ? b0 + sh.rp[k] : grp[k];
                    to[b] = right ? rq : lq;
                    ev[b] = elp<W>(right ? lq : rq);
                }
            }
#pragma unroll
            for (int b = 0; b < kBatch; ++b)
                if (k0 + (uint32_t)(kRT * b) < ks) store(to[b], ev[b]);
        }
        if (W != kSrc && tid == 0) {  // in place: the median-of-three swap, unless its slot is a swap target
            if (first >= nf && first < nl) store(first, pv.e);
            if (pv.ch >= nf && pv.ch < nl) {
                const uint32_t s = (pv.ch - b0) / 64, bit = (pv.ch - b0) % 64;
                const uint64_t below = low_mask(bit);
                bool tgt = false;
                if (!right && ((mge[s] >> bit) & 1ull)) tgt = gpre[s] + (uint32_t)__popcll(mge[s] & below) + 1 <= ks;
                if (right && ((mle[s] >> bit) & 1ull)) tgt = lsuf[s] - (uint32_t)__popcll(mle[s] & below) <= ks;
                if (!tgt) store(pv.ch, pv.f0);
            }
        }
        where = dst;
        base = nb;
        __syncthreads();
        phase(5);
        rec = rec || cut == nth;
        first = nf;
        last = nl;
    }

    template <int P, int W>
    __device__ __forceinline__ void round_any() {
        const uint32_t ns = (last - (first & ~63u) + 63) / 64;
        if (W == kLds || ns <= (uint32_t)kMeta) round<P, W, true>();
        else round<P, W, false>();
    }

    // ---------------------------------------------------------------- heap select (depth limit), one lane
    // stl_heap.h __adjust_heap / __push_heap / __make_heap / __pop_heap and stl_algo.h __heap_select,
    // restated over positions first + i (tests/cpp/introselect_model.cpp checks the restatement)
    template <int P>
    __device__ __forceinline__ void push_heap(uint32_t hole, uint32_t top, El value) {
        uint32_t parent = (hole - 1) / 2;
        while (hole > top && less<P>(get_any(first + parent), value)) {
            put_any(first + hole, get_any(first + parent));
            hole = parent;
            parent = (hole - 1) / 2;
        }
        put_any(first + hole, value);
    }
    template <int P>
    __device__ __forceinline__ void adjust_heap(uint32_t hole, uint32_t len, El value) {
        const uint32_t top = hole;
        uint32_t second = hole;
        while (len >= 1 && second < (len - 1) / 2) {
            second = 2 * (second + 1);
            if (less<P>(get_any(first + second), get_any(first + second - 1))) second--;
            put_any(first + hole, get_any(first + second));
            hole = second;
        }
        if ((len & 1u) == 0 && second == (len - 2) / 2) {
            second = 2 * (second + 1);
            put_any(first + hole, get_any(first + second - 1));
            hole = second - 1;
        }
        push_heap<P>(hole, top, value);
    }
    template <int P>
    __device__ __forceinline__ void heap_select(uint32_t middle, uint32_t len) {
        if (middle >= 2) {
            uint32_t parent = (middle - 2) / 2;
            while (true) {
                adjust_heap<P>(parent, middle, get_any(first + parent));
                if (parent == 0) break;
                parent--;
            }
        }
        for (uint32_t i = middle; i < len; ++i)
            if (less<P>(get_any(first + i), get_any(first))) {
                const El v = get_any(first + i);
                put_any(first + i, get_any(first));
                adjust_heap<P>(0, middle, v);
            }
    }

    // ---------------------------------------------------------------- std::nth_element(vec, vec + nth)
    // returns (vec[nth - 1], vec[nth]) of the post-state as values (lo only when nth >= 1), on thread 0
    template <int P>
    __device__ __forceinline__ void select(double& lo, double& hi) {
        first = 0; last = M; base = 0; where = kSrc; rec = 0;
        depth = M > 1 ? 2 * lg2(M) : 0;
        const uint64_t t0 = clock64();
        uint32_t nglb = 0, nlds = 0;
        if (last - first > 3) {
            --depth;
            round_any<P, kSrc>();
        }
        const uint64_t t1 = clock64();
        while (last - first > 3) {
            if (depth == 0) {
                if (tid == 0) {
                    heap_select<P>(nth + 1 - first, last - first);
                    const El f0 = get_any(first), n0 = get_any(nth);
                    put_any(first, n0);
                    put_any(nth, f0);
                }
                __syncthreads();
                break;
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
            if (where == kLds) { round_any<P, kLds>(); ++nlds; }
            else { round_any<P, kGlb>(); ++nglb; }
        }
        if (tid == 0) {
            sh.stamp[4 * P] = t1 - t0;
            sh.stamp[4 * P + 1] = clock64() - t1;
            sh.stamp[4 * P + 2] = nglb;
            sh.stamp[4 * P + 3] = nlds;
            if (last - first <= 3) {  // std::__insertion_sort of the last <= 3
                const uint32_t n = last - first;
                El v[3];
                for (uint32_t i = 0; i < n; ++i) v[i] = get_any(first + i);
                for (uint32_t i = 1; i < n; ++i) {
                    const El x = v[i];
                    uint32_t j = i;
                    while (j > 0 && less<P>(x, v[j - 1])) { v[j] = v[j - 1]; --j; }
                    v[j] = x;
                }
                for (uint32_t i = 0; i < n; ++i) sh.fin[i] = v[i];
                hi = value<P>(sh.fin[nth - first]);
                if (nth >= 1) lo = value<P>(rec ? lo_el : sh.fin[nth - 1 - first]);
            } else {  // heap select ran
                hi = value<P>(get_any(nth));
                if (nth >= 1) lo = value<P>(rec ? lo_el : get_any(nth - 1));
            }
        }
    }
};

// computeMedian / computeMAD (src/algorithm.cpp:834-865) with the reference's post-state: thread 0 of the
// block gets med and mad.  M slots, n visible.
template <typename Id, class Src>
__device__ __forceinline__ void ref_robust_scale(const Src& src, RefShared<Id>& sh, uint32_t* sel, int64_t sel_stride,
                                                 uint32_t M, uint32_t n, double& med, double& mad) {
    const int tid = (int)threadIdx.x;
    RefSel<Src, Id> s{src, sh};
    const int64_t q = sel_stride / 4;  // q >= M entries each: keys, ids, then the big segments' step records
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
    s.tid = tid; s.lane = tid & 63; s.wave = tid >> 6;
    s.med = 0.0;
    const bool even = (M & 1u) == 0 && s.nth >= 1;  // mid == 0 (UB in the reference) reads vec[mid]
    double lo = 0.0, hi = 0.0;
    s.template select<0>(lo, hi);
    __shared__ double bc;
    if (tid == 0) bc = even ? (lo + hi) / 2.0 : hi;
    __syncthreads();
    s.med = bc;
    s.template select<1>(lo, hi);
    if (tid == 0) {
        med = bc;
        mad = even ? (lo + hi) / 2.0 : hi;
    }
    __syncthreads();
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
        ref_robust_scale<Id>(src, sh, a.sel + (int64_t)pair * a.sel_stride, a.sel_stride, M, n, med, mad);
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
    (void)flags;
    __syncthreads();
    ArrSrc src{v};
    double med = 0.0, mad = 0.0;
    ref_robust_scale<Id>(src, sh, sel, sel_stride, M, n, med, mad);
    if (threadIdx.x == 0) {
        out[0] = med;
        out[1] = mad;
        for (int i = 0; i < 26; ++i) out[2 + i] = (double)sh.stamp[i];
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
