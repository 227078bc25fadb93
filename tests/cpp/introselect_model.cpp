// introselect_model.cpp — host model of the round formulation K2R (csrc/align.hip, median_mode
// SVO_MEDIAN_REFERENCE) uses to reproduce libstdc++'s std::nth_element on the device, checked against the
// real std::nth_element of this toolchain (test infrastructure; tests/test_introselect_model.py builds and
// runs it).
//
// The reference's robust scale reads vec[mid - 1] after std::nth_element(vec, mid) on the full residual
// vector (src/algorithm.cpp:834-853), i.e. whatever libstdc++'s introselect left there.  The device cannot
// run the sequential Hoare loop, so each partition round is restated in a form made of counts, prefix
// sums and maxima over the segment:
//
//   move_median_to_first(first, first+1, first+S/2, last-1), pivot p = a[first]        (stl_algo.h)
//   GE = positions i in [first+1, last) with !(a[i] < p), left to right: L_1 < L_2 < ...
//   LE = positions i in [first,   last) with !(p < a[i]), right to left: R_1 > R_2 > ...
//        (position first holds p: the right scan's sentinel)
//   __unguarded_partition swaps a[L_k] <-> a[R_k] exactly for k = 1 .. Ks, where
//        Ks = max over split points t in [first+1, last] of min(#GE before t, #LE from t on)
//   and returns cut = min(L_{Ks+1}, R_{Ks})   (R_0 = +inf; L_{Ks+1} = +inf when it does not exist).
//
// Proof sketch: the left scan of the k-th iteration starts after L_{k-1} and meets only original values
// until R_{k-1}, which now holds a value >= p; symmetrically for the right scan.  So while L_k < R_k the
// scans stop at the original L_k, R_k and swap them, and the first k with L_k >= R_k ends the loop at
// min(L_k, R_{k-1}).  L_k < R_k  <=>  some split t has L_k < t <= R_k  <=>  #GE before t >= k and #LE
// from t >= k, hence Ks.
//
// This program runs the model and std::nth_element on many inputs (random values, heavy duplicates,
// DBL_MAX padding like the reference's invisible residuals, every size up to 40, and median-of-3
// "killer" inputs built with McIlroy's adversary so that the depth limit forces the heap-select path)
// and requires the whole final array to be identical, plus the (vec[mid-1], vec[mid]) pair from the
// early-recording variant the device uses.  Prints "ok <cases>" or the first mismatch.
// "introselect_model killer N NTH FILE" writes the adversary's N doubles for nth = NTH (GPU test input).
#include <algorithm>
#include <cfloat>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <vector>

using V = double;

// ---- heap select, restated (stl_heap.h __adjust_heap / __push_heap / __make_heap / __pop_heap,
// stl_algo.h __heap_select): only reached when the depth limit runs out
static void push_heap_m(V* a, long hole, long top, V value) {
    long parent = (hole - 1) / 2;
    while (hole > top && a[parent] < value) {
        a[hole] = a[parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    a[hole] = value;
}
static void adjust_heap_m(V* a, long hole, long len, V value) {
    const long top = hole;
    long second = hole;
    while (second < (len - 1) / 2) {
        second = 2 * (second + 1);
        if (a[second] < a[second - 1]) second--;
        a[hole] = a[second];
        hole = second;
    }
    if ((len & 1) == 0 && second == (len - 2) / 2) {
        second = 2 * (second + 1);
        a[hole] = a[second - 1];
        hole = second - 1;
    }
    push_heap_m(a, hole, top, value);
}
static void make_heap_m(V* a, long len) {
    if (len < 2) return;
    long parent = (len - 2) / 2;
    while (true) {
        adjust_heap_m(a, parent, len, a[parent]);
        if (parent == 0) return;
        parent--;
    }
}
static void heap_select_m(V* first, long middle, long last) {
    make_heap_m(first, middle);
    for (long i = middle; i < last; ++i)
        if (first[i] < first[0]) {  // __pop_heap(first, middle, i)
            const V value = first[i];
            first[i] = first[0];
            adjust_heap_m(first, 0, middle, value);
        }
}

// ---- one round in the parallel form; returns cut, swaps applied in place
static long round_pf(std::vector<V>& a, long first, long last) {
    const long S = last - first, m = first + S / 2;
    const long A = first + 1, B = m, C = last - 1;
    long ch;
    if (a[A] < a[B]) ch = a[B] < a[C] ? B : (a[A] < a[C] ? C : A);
    else ch = a[A] < a[C] ? A : (a[B] < a[C] ? C : B);
    std::swap(a[first], a[ch]);
    const V p = a[first];
    // counts per position; G(t) = #GE in [first+1, t), Lc(t) = #LE in [t, last)
    std::vector<long> ge, le;  // L_1.., R_1..
    for (long i = first + 1; i < last; ++i)
        if (!(a[i] < p)) ge.push_back(i);
    for (long i = last - 1; i >= first; --i)
        if (!(p < a[i])) le.push_back(i);
    long total_le = (long)le.size();
    long ks = 0, g = 0, lc = total_le - (!(p < a[first]) ? 1 : 0);  // t = first + 1
    for (long t = first + 1; t <= last; ++t) {
        ks = std::max(ks, std::min(g, lc));
        if (t < last) {
            if (!(a[t] < p)) ++g;
            if (!(p < a[t])) --lc;
        }
    }
    long cut = (long)ge.size() > ks ? ge[ks] : LONG_MAX;
    if (ks > 0) cut = std::min(cut, le[ks - 1]);
    for (long k = 0; k < ks; ++k) std::swap(a[ge[k]], a[le[k]]);
    return cut;
}

static int lg(long n) { int r = 0; while (n >>= 1) ++r; return r; }

// the model of std::nth_element(a, a + nth, a + n).  lo_rec: the value the device reports for
// vec[nth - 1] (recorded at the round that cuts exactly at nth, else read after the final sort)
static void nth_model(std::vector<V>& a, long nth, V* lo_rec, bool* heap_used) {
    long first = 0, last = (long)a.size();
    *heap_used = false;
    bool rec = false;
    if (first == last || nth == last) return;
    int depth = 2 * lg(last - first);
    while (last - first > 3) {
        if (depth == 0) {
            heap_select_m(a.data() + first, nth + 1 - first, last - first);
            std::swap(a[first], a[nth]);
            *heap_used = true;
            if (!rec && nth >= 1) *lo_rec = a[nth - 1];
            return;
        }
        --depth;
        const long cut = round_pf(a, first, last);
        if (cut == nth && !rec && nth >= 1) { *lo_rec = a[nth - 1]; rec = true; }
        if (cut <= nth) first = cut;
        else last = cut;
    }
    std::sort(a.begin() + first, a.begin() + last);  // insertion sort of <= 3 values: same multiset order
    if (!rec && nth >= 1) *lo_rec = a[nth - 1];
}

// ---- McIlroy's adversary: values fixed lazily so that std::nth_element degenerates
static std::vector<V> killer(long n, long nth) {
    std::vector<long> val(n), ptr(n);
    const long gas = n;
    long nsolid = 0, candidate = 0;
    for (long i = 0; i < n; ++i) { val[i] = gas; ptr[i] = i; }
    auto cmp = [&](long x, long y) {
        if (val[x] == gas && val[y] == gas) {
            if (x == candidate) val[x] = nsolid++;
            else val[y] = nsolid++;
        }
        if (val[x] == gas) candidate = x;
        else if (val[y] == gas) candidate = y;
        return val[x] < val[y];
    };
    std::nth_element(ptr.begin(), ptr.begin() + nth, ptr.end(), cmp);
    std::vector<V> out(n);
    for (long i = 0; i < n; ++i) out[i] = (V)val[i];
    return out;
}

static long g_cases = 0, g_heap = 0;
static bool check(const std::vector<V>& in, long nth, const char* what) {
    std::vector<V> ref(in), mod(in);
    if (nth < (long)in.size()) std::nth_element(ref.begin(), ref.begin() + nth, ref.end());
    V lo = 0;
    bool heap = false;
    if (nth < (long)in.size()) nth_model(mod, nth, &lo, &heap);
    ++g_cases;
    g_heap += heap;
    if (ref != mod) {
        std::printf("MISMATCH %s n=%zu nth=%ld (array)\n", what, in.size(), nth);
        return false;
    }
    if (nth >= 1 && nth < (long)in.size() && !(lo == ref[nth - 1])) {
        std::printf("MISMATCH %s n=%zu nth=%ld (recorded lo %.17g vs %.17g)\n", what, in.size(), nth, lo, ref[nth - 1]);
        return false;
    }
    return true;
}

int main(int argc, char** argv) {
    if (argc == 5 && std::string(argv[1]) == "killer") {  // write an adversarial input (doubles) to argv[4]
        const std::vector<V> v = killer(std::atol(argv[2]), std::atol(argv[3]));
        FILE* f = std::fopen(argv[4], "wb");
        if (!f || std::fwrite(v.data(), sizeof(V), v.size(), f) != v.size()) return 3;
        std::fclose(f);
        return 0;
    }
    const long trials = argc > 1 ? std::atol(argv[1]) : 2000;
    std::mt19937_64 rng(12345);
    // every small size and every nth
    for (long n = 1; n <= 40; ++n)
        for (long nth = 0; nth < n; ++nth)
            for (int rep = 0; rep < 6; ++rep) {
                std::vector<V> v(n);
                for (auto& x : v) x = (V)(rng() % (rep < 3 ? 4 : 1000));
                if (!check(v, nth, "small")) return 1;
            }
    for (long t = 0; t < trials; ++t) {
        const long n = 4 + (long)(rng() % (t % 10 == 0 ? 60000 : 3000));
        const int kind = (int)(t % 5);
        std::vector<V> v(n);
        std::normal_distribution<double> nd(0.0, 8.0);
        long nvis = n;
        for (long i = 0; i < n; ++i) {
            switch (kind) {
                case 0: v[i] = nd(rng); break;                                  // distinct residuals
                case 1: v[i] = std::round(nd(rng)); break;                      // heavy ties
                case 2: v[i] = (double)(rng() % 3); break;                      // three values
                default: v[i] = nd(rng); break;
            }
        }
        if (kind >= 3) {  // invisible slots = DBL_MAX, in whole patches of 25 like the reference's features
            nvis = 0;
            const double pv = kind == 3 ? 0.8 : 0.3;
            for (long f = 0; f * 25 < n; ++f) {
                const bool vis = std::uniform_real_distribution<double>(0, 1)(rng) < pv;
                for (long k = f * 25; k < std::min(n, f * 25 + 25); ++k) {
                    if (!vis) v[k] = DBL_MAX;
                    else ++nvis;
                }
            }
        }
        const long nth = kind >= 3 ? nvis / 2 : (long)(rng() % n);
        if (nth >= n) continue;
        if (!check(v, nth, "random")) return 1;
        // the MAD pass: |v - med| in the original order (DBL_MAX stays DBL_MAX)
        if (kind >= 3 && nvis > 0) {
            std::vector<V> c(v);
            std::nth_element(c.begin(), c.begin() + nth, c.end());
            const double med = (n % 2 || nth == 0) ? c[nth] : (c[nth - 1] + c[nth]) / 2.0;
            std::vector<V> d(n);
            for (long i = 0; i < n; ++i) d[i] = std::fabs(v[i] - med);
            if (!check(d, nth, "mad")) return 1;
        }
    }
    // adversarial inputs: the depth limit runs out (heap-select path)
    for (long n : {200L, 1000L, 5000L, 50000L})
        for (long nth : {n / 2, n / 3, n - 1, 1L}) {
            std::vector<V> v = killer(n, nth);
            if (!check(v, nth, "killer")) return 1;
        }
    std::printf("ok %ld cases (%ld took the heap-select path)\n", g_cases, g_heap);
    return g_heap > 0 ? 0 : 2;
}
