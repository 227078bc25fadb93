// sort_check.cpp — the product's keypoint sort (svo::feature_sort_keys, libsvo_hip.so) against the real
// libstdc++ std::sort with the reference's comparator (src/feature_selection.cpp:53-54) on many inputs:
// the permutations must be identical.  Built and run by tests/test_feature_selection.py (no GPU needed).
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <random>
#include <vector>

namespace svo {
void feature_sort_keys(uint32_t* keys, int32_t n);
}

int main() {
    std::mt19937 rng(12345);
    int cases = 0;
    const int sizes[] = {0, 1, 2, 3, 5, 16, 17, 18, 33, 100, 1000, 4097, 20000, 40000, 71186, 150000};
    for (int n : sizes) {
        for (int dist = 0; dist < 7; ++dist) {
            std::vector<uint32_t> v(n);
            for (int i = 0; i < n; ++i) {
                uint32_t r = 0;
                switch (dist) {
                    case 0: r = rng() & 255; break;                                        // uniform
                    case 1: r = 51 + (uint32_t)std::min(204.0, std::exponential_distribution<double>(1.0 / 30)(rng)); break;
                    case 2: r = 7; break;                                                  // all equal
                    case 3: r = (uint32_t)(i * 256LL / (n + 1)); break;                    // ascending
                    case 4: r = 255 - (uint32_t)(i * 256LL / (n + 1)); break;              // descending
                    case 5: r = rng() % 3; break;                                          // three values
                    default: r = (i % 2) ? 200 : (rng() & 255); break;                     // half ties
                }
                v[i] = (r << 24) | (uint32_t)i;
            }
            std::vector<uint32_t> a = v, b = v;
            std::sort(a.begin(), a.end(), [](uint32_t x, uint32_t y) { return (x >> 24) > (y >> 24); });
            svo::feature_sort_keys(b.data(), n);
            if (a != b) {
                std::printf("MISMATCH n=%d dist=%d\n", n, dist);
                return 1;
            }
            ++cases;
        }
    }
    std::printf("ok %d cases\n", cases);
    return 0;
}
