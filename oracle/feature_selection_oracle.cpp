// =====================================================================================================
//  feature_selection_oracle.cpp — CPU restatement of the reference's FeatureSelection.
//
//  TEST INFRASTRUCTURE ONLY (same rules as svo_oracle.cpp): loaded by tests/ and bench.py's
//  cpu_baseline leg as the checker; the product never links or calls it.
//
//  Restates (paths relative to the reference root):
//    FeatureSelection ctor ............ src/feature_selection.cpp:19-25 (grid (H/c+1) x (W/c+1))
//    gradientMagnitudeWithSSC ......... src/feature_selection.cpp:27-89
//    gradientMagnitudeByValue ......... src/feature_selection.cpp:91-164 (bucketing branch)
//    SSC .............................. src/feature_selection.cpp:166-248
//    computeImageGradient ............. src/feature_selection.cpp:250-266 (orientation stays 0)
//    setExistingFeatures / setCell.. .. src/feature_selection.cpp:268-282, resetGridOccupancy :284-287
//  The keypoint record is laid out like cv::KeyPoint (pt, size, angle, response, octave, class_id)
//  and sorted with the reference's comparator by the real libstdc++ std::sort, so ties in the response
//  come out in the order that toolchain's introsort leaves them (the reference's own order on a
//  libstdc++ build).
//
//  One defined reading where the reference is undefined: when SSC's binary search reaches width 0
//  (fewer than Kmin keypoints), `c = width / 2.0` is 0 and the reference divides by zero and sizes a
//  vector from INT_MIN (std::length_error).  Here the search stops there and returns the previous
//  iteration's result, as its `low > high` exit does.
// =====================================================================================================
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <vector>

namespace fs_oracle {

struct KeyPoint {  // cv::KeyPoint(cv::Point2i(j, i), 1.0, angle, response)
    float x, y, size, angle, response;
    int octave, class_id;
};

// Simd::AbsGradientSaturatedSum (3rd_party/simd/include/Simd/SimdLib.h:856-884), border = 0
static void abs_gradient(const uint8_t* img, int w, int h, std::vector<uint8_t>& g) {
    g.assign((size_t)w * h, 0);
    for (int y = 1; y < h - 1; ++y)
        for (int x = 1; x < w - 1; ++x) {
            const uint8_t* p = img + (size_t)y * w + x;
            const int s = std::abs(int(p[1]) - int(p[-1])) + std::abs(int(p[w]) - int(p[-w]));
            g[(size_t)y * w + x] = (uint8_t)std::min(s, 255);
        }
}

// FeatureSelection::SSC (src/feature_selection.cpp:166-248)
static void ssc(const std::vector<KeyPoint>& kps, int32_t numRetPoints, float tolerance, int32_t cols, int32_t rows,
                std::vector<int32_t>& resultVec) {
    int32_t exp1 = rows + cols + 2 * numRetPoints;
    long long exp2 = ((long long)4 * cols + (long long)4 * numRetPoints + (long long)4 * rows * numRetPoints +
                      (long long)rows * rows + (long long)cols * cols - (long long)2 * rows * cols +
                      (long long)4 * rows * cols * numRetPoints);
    double exp3 = std::sqrt(static_cast<double>(exp2));
    double exp4 = (2 * (numRetPoints - 1));
    double sol1 = -std::round((exp1 + exp3) / exp4);
    double sol2 = -std::round((exp1 - exp3) / exp4);
    int high = (sol1 > sol2) ? static_cast<int>(sol1) : static_cast<int>(sol2);
    int low = static_cast<int>(std::sqrt((double)kps.size() / numRetPoints));
    int width;
    int prevWidth = -1;
    bool complete = false;
    float K = static_cast<float>(numRetPoints);
    uint32_t Kmin = static_cast<uint32_t>(std::round(K - (K * tolerance)));
    uint32_t Kmax = static_cast<uint32_t>(std::round(K + (K * tolerance)));
    std::vector<int32_t> result;
    result.reserve(kps.size());
    while (!complete) {
        width = low + (high - low) / 2;
        if (width == prevWidth || low > high || width <= 0) {  // width <= 0: see the header
            resultVec = result;
            break;
        }
        result.clear();
        double c = width / 2.0;
        int32_t numCellCols = static_cast<int32_t>(cols / c);
        int32_t numCellRows = static_cast<int32_t>(rows / c);
        std::vector<std::vector<bool>> coveredVec(numCellRows + 1, std::vector<bool>(numCellCols + 1, false));
        for (unsigned int i = 0; i < kps.size(); ++i) {
            int32_t row = static_cast<int32_t>(kps[i].y / c);
            int32_t col = static_cast<int32_t>(kps[i].x / c);
            if (coveredVec[row][col] == false) {
                result.push_back(i);
                const int32_t k = static_cast<int32_t>(width / c);
                int32_t rowMin = row >= k ? (row - k) : 0;
                int32_t rowMax = ((row + k) <= numCellRows) ? (row + k) : numCellRows;
                int32_t colMin = col >= k ? (col - k) : 0;
                int32_t colMax = ((col + k) <= numCellCols) ? (col + k) : numCellCols;
                for (int32_t r = rowMin; r <= rowMax; ++r)
                    for (int32_t cc = colMin; cc <= colMax; ++cc)
                        if (!coveredVec[r][cc]) coveredVec[r][cc] = true;
            }
        }
        if (result.size() >= Kmin && result.size() <= Kmax) {
            resultVec = result;
            complete = true;
        } else if (result.size() < Kmin)
            high = width - 1;
        else
            low = width + 1;
        prevWidth = width;
    }
}

struct Selector {  // FeatureSelection (src/feature_selection.cpp:19-25)
    int32_t cellSize, gridRows, gridCols;
    std::vector<bool> grid;
    Selector(int32_t w, int32_t h, int32_t c)
        : cellSize(c), gridRows(h / c + 1), gridCols(w / c + 1), grid((size_t)gridRows * gridCols, false) {}
    void setCell(double x, double y) {  // setCellInGridOccupancy (:276-282)
        uint32_t idx = x / cellSize;
        uint32_t idy = y / cellSize;
        grid[idy * gridCols + idx] = true;
    }
};

}  // namespace fs_oracle

using namespace fs_oracle;

extern "C" {

// The keypoint order of :53-54 (std::sort, reference comparator) for responses given in row-major
// keypoint order; perm[k] = row-major index of the k-th sorted keypoint.
void oracle_sort_responses(const uint8_t* resp, int32_t n, int32_t* perm) {
    std::vector<KeyPoint> kps(n);
    for (int32_t i = 0; i < n; ++i) kps[i] = {0.0f, 0.0f, 1.0f, 0.0f, (float)resp[i], 0, i};
    std::sort(kps.begin(), kps.end(), [](const KeyPoint& lhs, const KeyPoint& rhs) { return lhs.response > rhs.response; });
    for (int32_t i = 0; i < n; ++i) perm[i] = kps[i].class_id;
}

// SSC alone on keypoints already in sorted order (x, y of each); writes the selected indices.
int32_t oracle_ssc(const float* x, const float* y, int32_t n, int32_t num_ret, float tolerance, int32_t cols,
                   int32_t rows, int32_t* out) {
    std::vector<KeyPoint> kps(n);
    for (int32_t i = 0; i < n; ++i) kps[i] = {x[i], y[i], 1.0f, 0.0f, 0.0f, 0, -1};
    std::vector<int32_t> res;
    ssc(kps, num_ret, tolerance, cols, rows, res);
    std::copy(res.begin(), res.end(), out);
    return (int32_t)res.size();
}

// gradientMagnitudeWithSSC(frame, threshold, numberCandidate, useBucketing) on one base image.
// occupancy: the selector's grid ((h/c+1)*(w/c+1) bytes, in/out: setExistingFeatures before, reset after
// the bucketing branch).  Out: the new features' pixel positions and responses in addFeature order;
// n_keypoints = keypoints above the threshold.  Returns the feature count (-1 if capacity is short).
int32_t oracle_feature_select_ssc(const uint8_t* img, int32_t w, int32_t h, int32_t threshold, int32_t num_candidates,
                                  int32_t use_bucketing, int32_t cell_size, uint8_t* occupancy, int32_t capacity,
                                  double* px_out, double* resp_out, int32_t* n_keypoints) {
    Selector sel(w, h, cell_size);
    for (size_t i = 0; i < sel.grid.size(); ++i) sel.grid[i] = occupancy[i] != 0;
    std::vector<uint8_t> mag;
    abs_gradient(img, w, h, mag);
    std::vector<KeyPoint> keyPoints;
    keyPoints.reserve(10 * num_candidates);
    for (int32_t i = 0; i < h; i++)
        for (int32_t j = 0; j < w; j++)
            if (mag[(size_t)i * w + j] > (uint32_t)threshold)
                keyPoints.push_back({(float)j, (float)i, 1.0f, 0.0f, (float)mag[(size_t)i * w + j], 0, -1});
    std::sort(keyPoints.begin(), keyPoints.end(),
              [](const KeyPoint& lhs, const KeyPoint& rhs) { return lhs.response > rhs.response; });
    *n_keypoints = (int32_t)keyPoints.size();
    std::vector<int32_t> resultVec;
    resultVec.reserve(keyPoints.size());
    ssc(keyPoints, num_candidates, 0.1f, w, h, resultVec);
    int32_t n = 0;
    for (unsigned int i = 0; i < resultVec.size(); i++) {
        const KeyPoint& kp = keyPoints[resultVec[i]];
        if (use_bucketing) {
            int32_t idx = static_cast<int32_t>(kp.x) / sel.cellSize;
            int32_t idy = static_cast<int32_t>(kp.y) / sel.cellSize;
            if (sel.grid[idy * sel.gridCols + idx]) continue;
            sel.grid[idy * sel.gridCols + idx] = true;
        }
        if (n >= capacity) return -1;
        px_out[2 * n] = kp.x;
        px_out[2 * n + 1] = kp.y;
        resp_out[n] = kp.response;
        ++n;
    }
    if (use_bucketing) std::fill(sel.grid.begin(), sel.grid.end(), false);
    for (size_t i = 0; i < sel.grid.size(); ++i) occupancy[i] = sel.grid[i];
    return n;
}

// gradientMagnitudeByValue(frame, threshold, useBucketing = true) (src/feature_selection.cpp:91-143).
int32_t oracle_feature_select_by_value(const uint8_t* img, int32_t w, int32_t h, int32_t threshold, int32_t cell_size,
                                       uint8_t* occupancy, int32_t capacity, double* px_out, double* resp_out) {
    Selector sel(w, h, cell_size);
    for (size_t i = 0; i < sel.grid.size(); ++i) sel.grid[i] = occupancy[i] != 0;
    std::vector<uint8_t> mag;
    abs_gradient(img, w, h, mag);
    int32_t n = 0;
    for (int32_t r = 0; r < sel.gridRows; r++)
        for (int32_t c = 0; c < sel.gridCols; c++) {
            if (sel.grid[r * sel.gridCols + c]) continue;
            const int32_t maxColIdx = (c + 1) * cell_size < w ? cell_size : w - (c * cell_size);
            const int32_t maxRowIdx = (r + 1) * cell_size < h ? cell_size : h - (r * cell_size);
            uint32_t max = 0;
            int32_t rowIdx = 0, colIdx = 0;
            for (int32_t i = 0; i < maxRowIdx; i++)
                for (int32_t j = 0; j < maxColIdx; j++) {
                    const uint8_t v = mag[(size_t)(r * cell_size + i) * w + c * cell_size + j];
                    if (v > max) {
                        rowIdx = r * cell_size + i;
                        colIdx = c * cell_size + j;
                        max = v;
                    }
                }
            if (max > (uint32_t)threshold) {
                if (n >= capacity) return -1;
                px_out[2 * n] = colIdx;
                px_out[2 * n + 1] = rowIdx;
                resp_out[n] = mag[(size_t)rowIdx * w + colIdx];
                ++n;
            }
        }
    std::fill(occupancy, occupancy + sel.grid.size(), 0);
    return n;
}

}  // extern "C"
