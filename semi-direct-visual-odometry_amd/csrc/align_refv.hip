// align_refv.hip — K2V: the reference's robust scale bit for bit with the residual vector resident in
// registers (median_mode SVO_MEDIAN_REFERENCE, vectors of up to kVCap slots; K2R in align_ref.hip takes
// larger ones).
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
// VGPRs each) holds the whole vector as R = 98 doubles per lane, and every round works on registers.
// Position q lives in lane q % 64 of wave (q / 64) % 8, row q / 512 ("step" q / 64 = 8 row + wave), so a
// segment [f, l) always spreads over all eight waves.  Per round:
//   1. classify (each wave its own steps): apply the median-of-three swap in registers, GE / LE by two
//      compares per step; the 64-bit masks go to LDS records;                       barrier
//   2. every wave scans the records of [f, l) (13 steps per lane), finds the crossing and Ks, then L_{Ks+1},
//      R_{Ks} and L_{Ks} by a counted step search + a bit select; the owners publish the pre-values the next
//      round's pivot and vec[nth - 1] need; sources write the mailbox (LDS, k - 1);  barrier
//   3. targets on the kept side take the mailbox values; all read the next pivot's candidates.
// A mailbox larger than kMbCap swaps runs in chunks.  Segments of <= 512 continue on one wave from an LDS
// copy without barriers; the depth limit falls back to the restated heap select (adversarial inputs only).
// No global traffic but the two reads of K1's residuals per pair and level (one per pass).
#include "svo_internal.h"
#include "svo_math.h"
#include "svo_wave.h"
#include "ref_common.h"

namespace svo {

namespace {

using namespace refsel;

constexpr int kVT = 512;              // threads per pair
constexpr int kVW = kVT / 64;         // waves
constexpr int kVRows = 98;            // doubles per lane: vectors of <= 50 176 slots
constexpr int kVBase = 80;            // first data VGPR (the asm blocks name v80 / v[80 + 2r])
constexpr int kVRegRows = 88;         // rows in v80..v255; rows 88..97 in LDS (VShared::lrow)
static_assert(kVBase + 2 * kVRegRows == 256, "register rows fill v80..v255");
constexpr uint32_t kVCap = (uint32_t)kVRows * kVT;
constexpr uint32_t kMbCap = 12288;    // mailbox (doubles); Ks beyond it exchanges in chunks
#ifndef SVO_ONEWAVE
#define SVO_ONEWAVE 512
#endif
constexpr uint32_t kOneWave = SVO_ONEWAVE;  // segments of <= kOneWave positions continue on wave 0
static_assert(kOneWave % 64 == 0 && kOneWave / 64 <= kVRegRows && 2 * kOneWave <= kMbCap, "one-wave segment rows");
// wave 0's register rows for the MAD pass, staged by the other waves during its one-wave rounds, past the one-wave
// segment and its mailbox
constexpr uint32_t kStage = 2 * kOneWave;
static_assert(kStage + 64 * kVRegRows <= kMbCap, "staging of wave 0's rows inside the mailbox");
#if defined(SVO_STAMPS)
constexpr int kScanGroup = 2;         // record reads the scan keeps in flight (the stamps cost registers)
#else
constexpr int kScanGroup = 4;
#endif

template <int R>
struct VShared {
    static constexpr int kSteps = R * kVW;
    // mailbox (mbx[0, kMbCap); the one-wave segment in [0, 512) and its mailbox in [512, 768)), then the
    // per-lane dummy slots of the branch-free exchange (mbx[kMbCap + lane]): one array, so a lane's slot is
    // one selected index
    double mbx[kMbCap + 64];
    uint4 rec[kSteps];                // per step of the round: GE lo, GE hi, LE lo, LE hi
    uint32_t pre[kSteps];             // per step: #GE | #LE << 16 before it (each wave writes its own steps)
    double pub[6];                    // pre-values published by their owners (candidates 0-3, record 4)
    uint32_t pubk[4];                 // the candidates' target ranks (0: not a target), by their owners
    double bcd;                       // broadcast of the median between the passes
    double lrow[R - kVRegRows][kVT];  // rows 88..97 of the vector (the rest is in registers)
    uint32_t tmp[2 * kVW];            // per-wave counts of the prologue
};

struct VDiag {  // svo_debug_robust_scale diagnostics
    uint32_t nblock[2], nwave[2], heap[2], nchunk[2];
    uint64_t cyc[2];
    uint64_t ph[12];  // thread 0's cycles per phase, both passes: load, classify, barrier 1, publish + side
                      // ranks, sources, barrier 2, targets, exits (dump, one-wave rounds, final), scan, crossing,
                      // searches
    uint32_t nlog;    // (stamps build) per block round: segment size and thread 0's cycles
    uint32_t log[64][2];
};
// a phase stamp of the debug kernel in the diagnostic build (make stamps: -DSVO_STAMPS, build/stamps/); in the
// regular build the stamps are compiled out (they cost the debug kernel registers below the VGPR fence)
#if defined(SVO_STAMPS_SMALL)  // (make stamps STAMPS_SMALL=1: the phases of block rounds of < 2048 positions only)
[[maybe_unused]] constexpr bool kStampsSmall = true;
#else
[[maybe_unused]] constexpr bool kStampsSmall = false;
#endif
#if defined(SVO_STAMPS)
#define VSTAMP(i) \
    do { \
        if (dg && tid == 0) { \
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

// The vector in registers.  Row r < 88 (positions 512 r + tid) of every lane lives in the VGPR pair
// v[80 + 2r : 81 + 2r] (v80..v255), outside the values the compiler allocates; rows 88..97 live in LDS.  The
// rows are loaded by one asm block (buffer loads straight into the pairs) and read / written by a
// block-uniform index in VGPR indexing mode (s_set_gpr_idx_on + v_mov).  The compiler's own code must stay in
// v0..v79: tools/check_vreg_fence.py checks the generated assembly at every build (the Makefile fails
// otherwise).  Left to the compiler, 98 register-resident doubles plus the round logic did not fit 256
// VGPRs: unrolled row bodies had their per-row values computed for all rows at once, and 16-double vectors
// indexed dynamically were copied whole at control-flow joins; both spilled to scratch, and the VGPR-count
// attribute does not cap the allocation.
#define SVO_VROWS_ASM \
    "v_add_u32 %[vt], 0x0, %[vo]\n\tbuffer_load_dwordx2 v[80:81], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x1000, %[vo]\n\tbuffer_load_dwordx2 v[82:83], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x2000, %[vo]\n\tbuffer_load_dwordx2 v[84:85], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x3000, %[vo]\n\tbuffer_load_dwordx2 v[86:87], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x4000, %[vo]\n\tbuffer_load_dwordx2 v[88:89], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x5000, %[vo]\n\tbuffer_load_dwordx2 v[90:91], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x6000, %[vo]\n\tbuffer_load_dwordx2 v[92:93], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x7000, %[vo]\n\tbuffer_load_dwordx2 v[94:95], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x8000, %[vo]\n\tbuffer_load_dwordx2 v[96:97], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x9000, %[vo]\n\tbuffer_load_dwordx2 v[98:99], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0xa000, %[vo]\n\tbuffer_load_dwordx2 v[100:101], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0xb000, %[vo]\n\tbuffer_load_dwordx2 v[102:103], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0xc000, %[vo]\n\tbuffer_load_dwordx2 v[104:105], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0xd000, %[vo]\n\tbuffer_load_dwordx2 v[106:107], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0xe000, %[vo]\n\tbuffer_load_dwordx2 v[108:109], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0xf000, %[vo]\n\tbuffer_load_dwordx2 v[110:111], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x10000, %[vo]\n\tbuffer_load_dwordx2 v[112:113], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x11000, %[vo]\n\tbuffer_load_dwordx2 v[114:115], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x12000, %[vo]\n\tbuffer_load_dwordx2 v[116:117], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x13000, %[vo]\n\tbuffer_load_dwordx2 v[118:119], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x14000, %[vo]\n\tbuffer_load_dwordx2 v[120:121], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x15000, %[vo]\n\tbuffer_load_dwordx2 v[122:123], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x16000, %[vo]\n\tbuffer_load_dwordx2 v[124:125], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x17000, %[vo]\n\tbuffer_load_dwordx2 v[126:127], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x18000, %[vo]\n\tbuffer_load_dwordx2 v[128:129], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x19000, %[vo]\n\tbuffer_load_dwordx2 v[130:131], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x1a000, %[vo]\n\tbuffer_load_dwordx2 v[132:133], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x1b000, %[vo]\n\tbuffer_load_dwordx2 v[134:135], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x1c000, %[vo]\n\tbuffer_load_dwordx2 v[136:137], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x1d000, %[vo]\n\tbuffer_load_dwordx2 v[138:139], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x1e000, %[vo]\n\tbuffer_load_dwordx2 v[140:141], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x1f000, %[vo]\n\tbuffer_load_dwordx2 v[142:143], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x20000, %[vo]\n\tbuffer_load_dwordx2 v[144:145], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x21000, %[vo]\n\tbuffer_load_dwordx2 v[146:147], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x22000, %[vo]\n\tbuffer_load_dwordx2 v[148:149], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x23000, %[vo]\n\tbuffer_load_dwordx2 v[150:151], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x24000, %[vo]\n\tbuffer_load_dwordx2 v[152:153], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x25000, %[vo]\n\tbuffer_load_dwordx2 v[154:155], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x26000, %[vo]\n\tbuffer_load_dwordx2 v[156:157], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x27000, %[vo]\n\tbuffer_load_dwordx2 v[158:159], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x28000, %[vo]\n\tbuffer_load_dwordx2 v[160:161], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x29000, %[vo]\n\tbuffer_load_dwordx2 v[162:163], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x2a000, %[vo]\n\tbuffer_load_dwordx2 v[164:165], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x2b000, %[vo]\n\tbuffer_load_dwordx2 v[166:167], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x2c000, %[vo]\n\tbuffer_load_dwordx2 v[168:169], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x2d000, %[vo]\n\tbuffer_load_dwordx2 v[170:171], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x2e000, %[vo]\n\tbuffer_load_dwordx2 v[172:173], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x2f000, %[vo]\n\tbuffer_load_dwordx2 v[174:175], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x30000, %[vo]\n\tbuffer_load_dwordx2 v[176:177], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x31000, %[vo]\n\tbuffer_load_dwordx2 v[178:179], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x32000, %[vo]\n\tbuffer_load_dwordx2 v[180:181], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x33000, %[vo]\n\tbuffer_load_dwordx2 v[182:183], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x34000, %[vo]\n\tbuffer_load_dwordx2 v[184:185], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x35000, %[vo]\n\tbuffer_load_dwordx2 v[186:187], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x36000, %[vo]\n\tbuffer_load_dwordx2 v[188:189], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x37000, %[vo]\n\tbuffer_load_dwordx2 v[190:191], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x38000, %[vo]\n\tbuffer_load_dwordx2 v[192:193], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x39000, %[vo]\n\tbuffer_load_dwordx2 v[194:195], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x3a000, %[vo]\n\tbuffer_load_dwordx2 v[196:197], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x3b000, %[vo]\n\tbuffer_load_dwordx2 v[198:199], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x3c000, %[vo]\n\tbuffer_load_dwordx2 v[200:201], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x3d000, %[vo]\n\tbuffer_load_dwordx2 v[202:203], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x3e000, %[vo]\n\tbuffer_load_dwordx2 v[204:205], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x3f000, %[vo]\n\tbuffer_load_dwordx2 v[206:207], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x40000, %[vo]\n\tbuffer_load_dwordx2 v[208:209], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x41000, %[vo]\n\tbuffer_load_dwordx2 v[210:211], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x42000, %[vo]\n\tbuffer_load_dwordx2 v[212:213], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x43000, %[vo]\n\tbuffer_load_dwordx2 v[214:215], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x44000, %[vo]\n\tbuffer_load_dwordx2 v[216:217], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x45000, %[vo]\n\tbuffer_load_dwordx2 v[218:219], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x46000, %[vo]\n\tbuffer_load_dwordx2 v[220:221], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x47000, %[vo]\n\tbuffer_load_dwordx2 v[222:223], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x48000, %[vo]\n\tbuffer_load_dwordx2 v[224:225], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x49000, %[vo]\n\tbuffer_load_dwordx2 v[226:227], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x4a000, %[vo]\n\tbuffer_load_dwordx2 v[228:229], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x4b000, %[vo]\n\tbuffer_load_dwordx2 v[230:231], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x4c000, %[vo]\n\tbuffer_load_dwordx2 v[232:233], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x4d000, %[vo]\n\tbuffer_load_dwordx2 v[234:235], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x4e000, %[vo]\n\tbuffer_load_dwordx2 v[236:237], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x4f000, %[vo]\n\tbuffer_load_dwordx2 v[238:239], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x50000, %[vo]\n\tbuffer_load_dwordx2 v[240:241], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x51000, %[vo]\n\tbuffer_load_dwordx2 v[242:243], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x52000, %[vo]\n\tbuffer_load_dwordx2 v[244:245], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x53000, %[vo]\n\tbuffer_load_dwordx2 v[246:247], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x54000, %[vo]\n\tbuffer_load_dwordx2 v[248:249], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x55000, %[vo]\n\tbuffer_load_dwordx2 v[250:251], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x56000, %[vo]\n\tbuffer_load_dwordx2 v[252:253], %[vt], %[rs], 0 offen\n\t" \
    "v_add_u32 %[vt], 0x57000, %[vo]\n\tbuffer_load_dwordx2 v[254:255], %[vt], %[rs], 0 offen\n\t"

// the MAD pass's |x - med| on the data registers in place (src/algorithm.cpp:860-863): one subtraction and one
// sign clear per row, no index sessions (the same IEEE result as fabs(x - med))
#define SVO_VMAD_ASM \
    "v_add_f64 v[80:81], v[80:81], -%[m]\n\tv_and_b32 v81, 0x7fffffff, v81\n\t" \
    "v_add_f64 v[82:83], v[82:83], -%[m]\n\tv_and_b32 v83, 0x7fffffff, v83\n\t" \
    "v_add_f64 v[84:85], v[84:85], -%[m]\n\tv_and_b32 v85, 0x7fffffff, v85\n\t" \
    "v_add_f64 v[86:87], v[86:87], -%[m]\n\tv_and_b32 v87, 0x7fffffff, v87\n\t" \
    "v_add_f64 v[88:89], v[88:89], -%[m]\n\tv_and_b32 v89, 0x7fffffff, v89\n\t" \
    "v_add_f64 v[90:91], v[90:91], -%[m]\n\tv_and_b32 v91, 0x7fffffff, v91\n\t" \
    "v_add_f64 v[92:93], v[92:93], -%[m]\n\tv_and_b32 v93, 0x7fffffff, v93\n\t" \
    "v_add_f64 v[94:95], v[94:95], -%[m]\n\tv_and_b32 v95, 0x7fffffff, v95\n\t" \
    "v_add_f64 v[96:97], v[96:97], -%[m]\n\tv_and_b32 v97, 0x7fffffff, v97\n\t" \
    "v_add_f64 v[98:99], v[98:99], -%[m]\n\tv_and_b32 v99, 0x7fffffff, v99\n\t" \
    "v_add_f64 v[100:101], v[100:101], -%[m]\n\tv_and_b32 v101, 0x7fffffff, v101\n\t" \
    "v_add_f64 v[102:103], v[102:103], -%[m]\n\tv_and_b32 v103, 0x7fffffff, v103\n\t" \
    "v_add_f64 v[104:105], v[104:105], -%[m]\n\tv_and_b32 v105, 0x7fffffff, v105\n\t" \
    "v_add_f64 v[106:107], v[106:107], -%[m]\n\tv_and_b32 v107, 0x7fffffff, v107\n\t" \
    "v_add_f64 v[108:109], v[108:109], -%[m]\n\tv_and_b32 v109, 0x7fffffff, v109\n\t" \
    "v_add_f64 v[110:111], v[110:111], -%[m]\n\tv_and_b32 v111, 0x7fffffff, v111\n\t" \
    "v_add_f64 v[112:113], v[112:113], -%[m]\n\tv_and_b32 v113, 0x7fffffff, v113\n\t" \
    "v_add_f64 v[114:115], v[114:115], -%[m]\n\tv_and_b32 v115, 0x7fffffff, v115\n\t" \
    "v_add_f64 v[116:117], v[116:117], -%[m]\n\tv_and_b32 v117, 0x7fffffff, v117\n\t" \
    "v_add_f64 v[118:119], v[118:119], -%[m]\n\tv_and_b32 v119, 0x7fffffff, v119\n\t" \
    "v_add_f64 v[120:121], v[120:121], -%[m]\n\tv_and_b32 v121, 0x7fffffff, v121\n\t" \
    "v_add_f64 v[122:123], v[122:123], -%[m]\n\tv_and_b32 v123, 0x7fffffff, v123\n\t" \
    "v_add_f64 v[124:125], v[124:125], -%[m]\n\tv_and_b32 v125, 0x7fffffff, v125\n\t" \
    "v_add_f64 v[126:127], v[126:127], -%[m]\n\tv_and_b32 v127, 0x7fffffff, v127\n\t" \
    "v_add_f64 v[128:129], v[128:129], -%[m]\n\tv_and_b32 v129, 0x7fffffff, v129\n\t" \
    "v_add_f64 v[130:131], v[130:131], -%[m]\n\tv_and_b32 v131, 0x7fffffff, v131\n\t" \
    "v_add_f64 v[132:133], v[132:133], -%[m]\n\tv_and_b32 v133, 0x7fffffff, v133\n\t" \
    "v_add_f64 v[134:135], v[134:135], -%[m]\n\tv_and_b32 v135, 0x7fffffff, v135\n\t" \
    "v_add_f64 v[136:137], v[136:137], -%[m]\n\tv_and_b32 v137, 0x7fffffff, v137\n\t" \
    "v_add_f64 v[138:139], v[138:139], -%[m]\n\tv_and_b32 v139, 0x7fffffff, v139\n\t" \
    "v_add_f64 v[140:141], v[140:141], -%[m]\n\tv_and_b32 v141, 0x7fffffff, v141\n\t" \
    "v_add_f64 v[142:143], v[142:143], -%[m]\n\tv_and_b32 v143, 0x7fffffff, v143\n\t" \
    "v_add_f64 v[144:145], v[144:145], -%[m]\n\tv_and_b32 v145, 0x7fffffff, v145\n\t" \
    "v_add_f64 v[146:147], v[146:147], -%[m]\n\tv_and_b32 v147, 0x7fffffff, v147\n\t" \
    "v_add_f64 v[148:149], v[148:149], -%[m]\n\tv_and_b32 v149, 0x7fffffff, v149\n\t" \
    "v_add_f64 v[150:151], v[150:151], -%[m]\n\tv_and_b32 v151, 0x7fffffff, v151\n\t" \
    "v_add_f64 v[152:153], v[152:153], -%[m]\n\tv_and_b32 v153, 0x7fffffff, v153\n\t" \
    "v_add_f64 v[154:155], v[154:155], -%[m]\n\tv_and_b32 v155, 0x7fffffff, v155\n\t" \
    "v_add_f64 v[156:157], v[156:157], -%[m]\n\tv_and_b32 v157, 0x7fffffff, v157\n\t" \
    "v_add_f64 v[158:159], v[158:159], -%[m]\n\tv_and_b32 v159, 0x7fffffff, v159\n\t" \
    "v_add_f64 v[160:161], v[160:161], -%[m]\n\tv_and_b32 v161, 0x7fffffff, v161\n\t" \
    "v_add_f64 v[162:163], v[162:163], -%[m]\n\tv_and_b32 v163, 0x7fffffff, v163\n\t" \
    "v_add_f64 v[164:165], v[164:165], -%[m]\n\tv_and_b32 v165, 0x7fffffff, v165\n\t" \
    "v_add_f64 v[166:167], v[166:167], -%[m]\n\tv_and_b32 v167, 0x7fffffff, v167\n\t" \
    "v_add_f64 v[168:169], v[168:169], -%[m]\n\tv_and_b32 v169, 0x7fffffff, v169\n\t" \
    "v_add_f64 v[170:171], v[170:171], -%[m]\n\tv_and_b32 v171, 0x7fffffff, v171\n\t" \
    "v_add_f64 v[172:173], v[172:173], -%[m]\n\tv_and_b32 v173, 0x7fffffff, v173\n\t" \
    "v_add_f64 v[174:175], v[174:175], -%[m]\n\tv_and_b32 v175, 0x7fffffff, v175\n\t" \
    "v_add_f64 v[176:177], v[176:177], -%[m]\n\tv_and_b32 v177, 0x7fffffff, v177\n\t" \
    "v_add_f64 v[178:179], v[178:179], -%[m]\n\tv_and_b32 v179, 0x7fffffff, v179\n\t" \
    "v_add_f64 v[180:181], v[180:181], -%[m]\n\tv_and_b32 v181, 0x7fffffff, v181\n\t" \
    "v_add_f64 v[182:183], v[182:183], -%[m]\n\tv_and_b32 v183, 0x7fffffff, v183\n\t" \
    "v_add_f64 v[184:185], v[184:185], -%[m]\n\tv_and_b32 v185, 0x7fffffff, v185\n\t" \
    "v_add_f64 v[186:187], v[186:187], -%[m]\n\tv_and_b32 v187, 0x7fffffff, v187\n\t" \
    "v_add_f64 v[188:189], v[188:189], -%[m]\n\tv_and_b32 v189, 0x7fffffff, v189\n\t" \
    "v_add_f64 v[190:191], v[190:191], -%[m]\n\tv_and_b32 v191, 0x7fffffff, v191\n\t" \
    "v_add_f64 v[192:193], v[192:193], -%[m]\n\tv_and_b32 v193, 0x7fffffff, v193\n\t" \
    "v_add_f64 v[194:195], v[194:195], -%[m]\n\tv_and_b32 v195, 0x7fffffff, v195\n\t" \
    "v_add_f64 v[196:197], v[196:197], -%[m]\n\tv_and_b32 v197, 0x7fffffff, v197\n\t" \
    "v_add_f64 v[198:199], v[198:199], -%[m]\n\tv_and_b32 v199, 0x7fffffff, v199\n\t" \
    "v_add_f64 v[200:201], v[200:201], -%[m]\n\tv_and_b32 v201, 0x7fffffff, v201\n\t" \
    "v_add_f64 v[202:203], v[202:203], -%[m]\n\tv_and_b32 v203, 0x7fffffff, v203\n\t" \
    "v_add_f64 v[204:205], v[204:205], -%[m]\n\tv_and_b32 v205, 0x7fffffff, v205\n\t" \
    "v_add_f64 v[206:207], v[206:207], -%[m]\n\tv_and_b32 v207, 0x7fffffff, v207\n\t" \
    "v_add_f64 v[208:209], v[208:209], -%[m]\n\tv_and_b32 v209, 0x7fffffff, v209\n\t" \
    "v_add_f64 v[210:211], v[210:211], -%[m]\n\tv_and_b32 v211, 0x7fffffff, v211\n\t" \
    "v_add_f64 v[212:213], v[212:213], -%[m]\n\tv_and_b32 v213, 0x7fffffff, v213\n\t" \
    "v_add_f64 v[214:215], v[214:215], -%[m]\n\tv_and_b32 v215, 0x7fffffff, v215\n\t" \
    "v_add_f64 v[216:217], v[216:217], -%[m]\n\tv_and_b32 v217, 0x7fffffff, v217\n\t" \
    "v_add_f64 v[218:219], v[218:219], -%[m]\n\tv_and_b32 v219, 0x7fffffff, v219\n\t" \
    "v_add_f64 v[220:221], v[220:221], -%[m]\n\tv_and_b32 v221, 0x7fffffff, v221\n\t" \
    "v_add_f64 v[222:223], v[222:223], -%[m]\n\tv_and_b32 v223, 0x7fffffff, v223\n\t" \
    "v_add_f64 v[224:225], v[224:225], -%[m]\n\tv_and_b32 v225, 0x7fffffff, v225\n\t" \
    "v_add_f64 v[226:227], v[226:227], -%[m]\n\tv_and_b32 v227, 0x7fffffff, v227\n\t" \
    "v_add_f64 v[228:229], v[228:229], -%[m]\n\tv_and_b32 v229, 0x7fffffff, v229\n\t" \
    "v_add_f64 v[230:231], v[230:231], -%[m]\n\tv_and_b32 v231, 0x7fffffff, v231\n\t" \
    "v_add_f64 v[232:233], v[232:233], -%[m]\n\tv_and_b32 v233, 0x7fffffff, v233\n\t" \
    "v_add_f64 v[234:235], v[234:235], -%[m]\n\tv_and_b32 v235, 0x7fffffff, v235\n\t" \
    "v_add_f64 v[236:237], v[236:237], -%[m]\n\tv_and_b32 v237, 0x7fffffff, v237\n\t" \
    "v_add_f64 v[238:239], v[238:239], -%[m]\n\tv_and_b32 v239, 0x7fffffff, v239\n\t" \
    "v_add_f64 v[240:241], v[240:241], -%[m]\n\tv_and_b32 v241, 0x7fffffff, v241\n\t" \
    "v_add_f64 v[242:243], v[242:243], -%[m]\n\tv_and_b32 v243, 0x7fffffff, v243\n\t" \
    "v_add_f64 v[244:245], v[244:245], -%[m]\n\tv_and_b32 v245, 0x7fffffff, v245\n\t" \
    "v_add_f64 v[246:247], v[246:247], -%[m]\n\tv_and_b32 v247, 0x7fffffff, v247\n\t" \
    "v_add_f64 v[248:249], v[248:249], -%[m]\n\tv_and_b32 v249, 0x7fffffff, v249\n\t" \
    "v_add_f64 v[250:251], v[250:251], -%[m]\n\tv_and_b32 v251, 0x7fffffff, v251\n\t" \
    "v_add_f64 v[252:253], v[252:253], -%[m]\n\tv_and_b32 v253, 0x7fffffff, v253\n\t" \
    "v_add_f64 v[254:255], v[254:255], -%[m]\n\tv_and_b32 v255, 0x7fffffff, v255\n\t"

// wave 0's rows for the MAD pass from their LDS staging (stg[64 r + lane], byte offset 512 r from the lane's
// address) straight into the data registers
#define SVO_VLDS_ASM \
    "ds_read_b64 v[80:81], %[a] offset:0\n\t" \
    "ds_read_b64 v[82:83], %[a] offset:512\n\t" \
    "ds_read_b64 v[84:85], %[a] offset:1024\n\t" \
    "ds_read_b64 v[86:87], %[a] offset:1536\n\t" \
    "ds_read_b64 v[88:89], %[a] offset:2048\n\t" \
    "ds_read_b64 v[90:91], %[a] offset:2560\n\t" \
    "ds_read_b64 v[92:93], %[a] offset:3072\n\t" \
    "ds_read_b64 v[94:95], %[a] offset:3584\n\t" \
    "ds_read_b64 v[96:97], %[a] offset:4096\n\t" \
    "ds_read_b64 v[98:99], %[a] offset:4608\n\t" \
    "ds_read_b64 v[100:101], %[a] offset:5120\n\t" \
    "ds_read_b64 v[102:103], %[a] offset:5632\n\t" \
    "ds_read_b64 v[104:105], %[a] offset:6144\n\t" \
    "ds_read_b64 v[106:107], %[a] offset:6656\n\t" \
    "ds_read_b64 v[108:109], %[a] offset:7168\n\t" \
    "ds_read_b64 v[110:111], %[a] offset:7680\n\t" \
    "ds_read_b64 v[112:113], %[a] offset:8192\n\t" \
    "ds_read_b64 v[114:115], %[a] offset:8704\n\t" \
    "ds_read_b64 v[116:117], %[a] offset:9216\n\t" \
    "ds_read_b64 v[118:119], %[a] offset:9728\n\t" \
    "ds_read_b64 v[120:121], %[a] offset:10240\n\t" \
    "ds_read_b64 v[122:123], %[a] offset:10752\n\t" \
    "ds_read_b64 v[124:125], %[a] offset:11264\n\t" \
    "ds_read_b64 v[126:127], %[a] offset:11776\n\t" \
    "ds_read_b64 v[128:129], %[a] offset:12288\n\t" \
    "ds_read_b64 v[130:131], %[a] offset:12800\n\t" \
    "ds_read_b64 v[132:133], %[a] offset:13312\n\t" \
    "ds_read_b64 v[134:135], %[a] offset:13824\n\t" \
    "ds_read_b64 v[136:137], %[a] offset:14336\n\t" \
    "ds_read_b64 v[138:139], %[a] offset:14848\n\t" \
    "ds_read_b64 v[140:141], %[a] offset:15360\n\t" \
    "ds_read_b64 v[142:143], %[a] offset:15872\n\t" \
    "ds_read_b64 v[144:145], %[a] offset:16384\n\t" \
    "ds_read_b64 v[146:147], %[a] offset:16896\n\t" \
    "ds_read_b64 v[148:149], %[a] offset:17408\n\t" \
    "ds_read_b64 v[150:151], %[a] offset:17920\n\t" \
    "ds_read_b64 v[152:153], %[a] offset:18432\n\t" \
    "ds_read_b64 v[154:155], %[a] offset:18944\n\t" \
    "ds_read_b64 v[156:157], %[a] offset:19456\n\t" \
    "ds_read_b64 v[158:159], %[a] offset:19968\n\t" \
    "ds_read_b64 v[160:161], %[a] offset:20480\n\t" \
    "ds_read_b64 v[162:163], %[a] offset:20992\n\t" \
    "ds_read_b64 v[164:165], %[a] offset:21504\n\t" \
    "ds_read_b64 v[166:167], %[a] offset:22016\n\t" \
    "ds_read_b64 v[168:169], %[a] offset:22528\n\t" \
    "ds_read_b64 v[170:171], %[a] offset:23040\n\t" \
    "ds_read_b64 v[172:173], %[a] offset:23552\n\t" \
    "ds_read_b64 v[174:175], %[a] offset:24064\n\t" \
    "ds_read_b64 v[176:177], %[a] offset:24576\n\t" \
    "ds_read_b64 v[178:179], %[a] offset:25088\n\t" \
    "ds_read_b64 v[180:181], %[a] offset:25600\n\t" \
    "ds_read_b64 v[182:183], %[a] offset:26112\n\t" \
    "ds_read_b64 v[184:185], %[a] offset:26624\n\t" \
    "ds_read_b64 v[186:187], %[a] offset:27136\n\t" \
    "ds_read_b64 v[188:189], %[a] offset:27648\n\t" \
    "ds_read_b64 v[190:191], %[a] offset:28160\n\t" \
    "ds_read_b64 v[192:193], %[a] offset:28672\n\t" \
    "ds_read_b64 v[194:195], %[a] offset:29184\n\t" \
    "ds_read_b64 v[196:197], %[a] offset:29696\n\t" \
    "ds_read_b64 v[198:199], %[a] offset:30208\n\t" \
    "ds_read_b64 v[200:201], %[a] offset:30720\n\t" \
    "ds_read_b64 v[202:203], %[a] offset:31232\n\t" \
    "ds_read_b64 v[204:205], %[a] offset:31744\n\t" \
    "ds_read_b64 v[206:207], %[a] offset:32256\n\t" \
    "ds_read_b64 v[208:209], %[a] offset:32768\n\t" \
    "ds_read_b64 v[210:211], %[a] offset:33280\n\t" \
    "ds_read_b64 v[212:213], %[a] offset:33792\n\t" \
    "ds_read_b64 v[214:215], %[a] offset:34304\n\t" \
    "ds_read_b64 v[216:217], %[a] offset:34816\n\t" \
    "ds_read_b64 v[218:219], %[a] offset:35328\n\t" \
    "ds_read_b64 v[220:221], %[a] offset:35840\n\t" \
    "ds_read_b64 v[222:223], %[a] offset:36352\n\t" \
    "ds_read_b64 v[224:225], %[a] offset:36864\n\t" \
    "ds_read_b64 v[226:227], %[a] offset:37376\n\t" \
    "ds_read_b64 v[228:229], %[a] offset:37888\n\t" \
    "ds_read_b64 v[230:231], %[a] offset:38400\n\t" \
    "ds_read_b64 v[232:233], %[a] offset:38912\n\t" \
    "ds_read_b64 v[234:235], %[a] offset:39424\n\t" \
    "ds_read_b64 v[236:237], %[a] offset:39936\n\t" \
    "ds_read_b64 v[238:239], %[a] offset:40448\n\t" \
    "ds_read_b64 v[240:241], %[a] offset:40960\n\t" \
    "ds_read_b64 v[242:243], %[a] offset:41472\n\t" \
    "ds_read_b64 v[244:245], %[a] offset:41984\n\t" \
    "ds_read_b64 v[246:247], %[a] offset:42496\n\t" \
    "ds_read_b64 v[248:249], %[a] offset:43008\n\t" \
    "ds_read_b64 v[250:251], %[a] offset:43520\n\t" \
    "ds_read_b64 v[252:253], %[a] offset:44032\n\t" \
    "ds_read_b64 v[254:255], %[a] offset:44544\n\t"

// the lane's value in block-uniform row r / store x there.  Index mode writes M0; M0 is reserved to the
// compiler, which uses it nowhere in these kernels (checked with the fence).  Volatile asm keeps the row
// accesses in program order.
__device__ __forceinline__ double vget(int r) {
    uint32_t lo, hi;
    asm volatile(
        "s_set_gpr_idx_on %2, gpr_idx(SRC0)\n\tv_mov_b32 %0, v80\n\tv_mov_b32 %1, v81\n\ts_set_gpr_idx_off"
        : "=v"(lo), "=v"(hi)
        : "s"(__builtin_amdgcn_readfirstlane(2 * r)));
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ void vset(int r, double x) {
    const uint64_t u = __builtin_bit_cast(uint64_t, x);
    asm volatile(
        "s_set_gpr_idx_on %2, gpr_idx(DST)\n\tv_mov_b32 v80, %0\n\tv_mov_b32 v81, %1\n\ts_set_gpr_idx_off"
        :
        : "v"((uint32_t)u), "v"((uint32_t)(u >> 32)), "s"(__builtin_amdgcn_readfirstlane(2 * r)));
}
// the row compares straight on the data registers (SRC0 indexed; no copy): ge = !(x < p), le = !(p < x)
__device__ __forceinline__ void vcmp2(int r, double p, uint64_t& ge, uint64_t& le) {
    asm volatile(
        "s_set_gpr_idx_on %2, gpr_idx(SRC0)\n\tv_cmp_nlt_f64 %0, v[80:81], %3\n\tv_cmp_ngt_f64 %1, v[80:81], %3\n\t"
        "s_set_gpr_idx_off"
        : "=&s"(ge), "=&s"(le)
        : "s"(__builtin_amdgcn_readfirstlane(2 * r)), "s"(p));
}
__device__ __forceinline__ uint64_t vcmp_ge(int r, double p) {
    uint64_t m;
    asm volatile("s_set_gpr_idx_on %1, gpr_idx(SRC0)\n\tv_cmp_nlt_f64 %0, v[80:81], %2\n\ts_set_gpr_idx_off"
                 : "=s"(m)
                 : "s"(__builtin_amdgcn_readfirstlane(2 * r)), "s"(p));
    return m;
}
__device__ __forceinline__ uint64_t vcmp_le(int r, double p) {
    uint64_t m;
    asm volatile("s_set_gpr_idx_on %1, gpr_idx(SRC0)\n\tv_cmp_ngt_f64 %0, v[80:81], %2\n\ts_set_gpr_idx_off"
                 : "=s"(m)
                 : "s"(__builtin_amdgcn_readfirstlane(2 * r)), "s"(p));
    return m;
}
// the lanes of m take x in row r (DST and SRC0 indexed: the register itself is the kept value)
__device__ __forceinline__ void vsel(int r, double x, uint64_t m) {
    const uint64_t u = __builtin_bit_cast(uint64_t, x);
    asm volatile(
        "s_set_gpr_idx_on %3, gpr_idx(SRC0,DST)\n\tv_cndmask_b32 v80, v80, %0, %2\n\tv_cndmask_b32 v81, v81, %1, %2\n\t"
        "s_set_gpr_idx_off"
        :
        : "v"((uint32_t)u), "v"((uint32_t)(u >> 32)), "s"(m), "s"(__builtin_amdgcn_readfirstlane(2 * r)));
}
// four consecutive rows r..r+3 (r + 3 < 88) in one index session: independent compares / moves / selects, so
// their latencies overlap (a row at a time, a round spent ~200 cycles per row on dependent chains)
__device__ __forceinline__ void vcmp2x4(int r, double p, uint64_t (&ge)[4], uint64_t (&le)[4]) {
    asm volatile(
        "s_set_gpr_idx_on %8, gpr_idx(SRC0)\n\t"
        "v_cmp_nlt_f64 %0, v[80:81], %9\n\tv_cmp_ngt_f64 %1, v[80:81], %9\n\t"
        "v_cmp_nlt_f64 %2, v[82:83], %9\n\tv_cmp_ngt_f64 %3, v[82:83], %9\n\t"
        "v_cmp_nlt_f64 %4, v[84:85], %9\n\tv_cmp_ngt_f64 %5, v[84:85], %9\n\t"
        "v_cmp_nlt_f64 %6, v[86:87], %9\n\tv_cmp_ngt_f64 %7, v[86:87], %9\n\t"
        "s_set_gpr_idx_off"
        : "=&s"(ge[0]), "=&s"(le[0]), "=&s"(ge[1]), "=&s"(le[1]), "=&s"(ge[2]), "=&s"(le[2]), "=&s"(ge[3]), "=&s"(le[3])
        : "s"(__builtin_amdgcn_readfirstlane(2 * r)), "s"(p));
}
// kind 0: ge = !(x < p); kind 1: le = !(p < x)
template <int kKind>
__device__ __forceinline__ void vcmpx4(int r, double p, uint64_t (&m)[4]) {
    if constexpr (kKind == 0)
        asm volatile(
            "s_set_gpr_idx_on %4, gpr_idx(SRC0)\n\tv_cmp_nlt_f64 %0, v[80:81], %5\n\tv_cmp_nlt_f64 %1, v[82:83], %5\n\t"
            "v_cmp_nlt_f64 %2, v[84:85], %5\n\tv_cmp_nlt_f64 %3, v[86:87], %5\n\ts_set_gpr_idx_off"
            : "=&s"(m[0]), "=&s"(m[1]), "=&s"(m[2]), "=&s"(m[3])
            : "s"(__builtin_amdgcn_readfirstlane(2 * r)), "s"(p));
    else
        asm volatile(
            "s_set_gpr_idx_on %4, gpr_idx(SRC0)\n\tv_cmp_ngt_f64 %0, v[80:81], %5\n\tv_cmp_ngt_f64 %1, v[82:83], %5\n\t"
            "v_cmp_ngt_f64 %2, v[84:85], %5\n\tv_cmp_ngt_f64 %3, v[86:87], %5\n\ts_set_gpr_idx_off"
            : "=&s"(m[0]), "=&s"(m[1]), "=&s"(m[2]), "=&s"(m[3])
            : "s"(__builtin_amdgcn_readfirstlane(2 * r)), "s"(p));
}
__device__ __forceinline__ void vgetx4(int r, double (&x)[4]) {
    uint32_t a0, a1, a2, a3, a4, a5, a6, a7;
    asm volatile(
        "s_set_gpr_idx_on %8, gpr_idx(SRC0)\n\tv_mov_b32 %0, v80\n\tv_mov_b32 %1, v81\n\tv_mov_b32 %2, v82\n\t"
        "v_mov_b32 %3, v83\n\tv_mov_b32 %4, v84\n\tv_mov_b32 %5, v85\n\tv_mov_b32 %6, v86\n\tv_mov_b32 %7, v87\n\t"
        "s_set_gpr_idx_off"
        : "=v"(a0), "=v"(a1), "=v"(a2), "=v"(a3), "=v"(a4), "=v"(a5), "=v"(a6), "=v"(a7)
        : "s"(__builtin_amdgcn_readfirstlane(2 * r)));
    x[0] = __builtin_bit_cast(double, ((uint64_t)a1 << 32) | a0);
    x[1] = __builtin_bit_cast(double, ((uint64_t)a3 << 32) | a2);
    x[2] = __builtin_bit_cast(double, ((uint64_t)a5 << 32) | a4);
    x[3] = __builtin_bit_cast(double, ((uint64_t)a7 << 32) | a6);
}
__device__ __forceinline__ void vselx4(int r, const double (&x)[4], const uint64_t (&m)[4]) {
    const uint64_t u0 = __builtin_bit_cast(uint64_t, x[0]), u1 = __builtin_bit_cast(uint64_t, x[1]);
    const uint64_t u2 = __builtin_bit_cast(uint64_t, x[2]), u3 = __builtin_bit_cast(uint64_t, x[3]);
    asm volatile(
        "s_set_gpr_idx_on %12, gpr_idx(SRC0,DST)\n\t"
        "v_cndmask_b32 v80, v80, %0, %8\n\tv_cndmask_b32 v81, v81, %1, %8\n\t"
        "v_cndmask_b32 v82, v82, %2, %9\n\tv_cndmask_b32 v83, v83, %3, %9\n\t"
        "v_cndmask_b32 v84, v84, %4, %10\n\tv_cndmask_b32 v85, v85, %5, %10\n\t"
        "v_cndmask_b32 v86, v86, %6, %11\n\tv_cndmask_b32 v87, v87, %7, %11\n\t"
        "s_set_gpr_idx_off"
        :
        : "v"((uint32_t)u0), "v"((uint32_t)(u0 >> 32)), "v"((uint32_t)u1), "v"((uint32_t)(u1 >> 32)),
          "v"((uint32_t)u2), "v"((uint32_t)(u2 >> 32)), "v"((uint32_t)u3), "v"((uint32_t)(u3 >> 32)),
          "s"(m[0]), "s"(m[1]), "s"(m[2]), "s"(m[3]), "s"(__builtin_amdgcn_readfirstlane(2 * r)));
}
// the lanes of m take a, the others b: one v_cndmask on the SGPR mask (the compiler's form of
// ((m >> lane) & 1) ? a : b costs a 64-bit shift, an and and a compare per use)
__device__ __forceinline__ uint32_t lane_sel(uint64_t m, uint32_t a, uint32_t b) {
    uint32_t r;
    asm("v_cndmask_b32_e64 %0, %2, %1, %3" : "=v"(r) : "v"(a), "v"(b), "s"(m));
    return r;
}
// one step record (GE mask, LE mask) stored at LDS byte address addr + kOff: two 64-bit moves from the SGPR
// masks and two 8-B stores (the compiler's form: four 32-bit moves, an address move and a 16-B store)
template <int kOff>
__device__ __forceinline__ void rec_put(uint32_t addr, uint64_t ge, uint64_t le) {
    uint64_t tg, tl;
    asm volatile("v_mov_b64 %0, %3\n\tv_mov_b64 %1, %4\n\tds_write_b64 %2, %0 offset:%5\n\tds_write_b64 %2, %1 offset:%6"
                 : "=&v"(tg), "=&v"(tl)
                 : "v"(addr), "s"(ge), "s"(le), "i"(kOff), "i"(kOff + 8)
                 : "memory");
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
// rows 0..87 of src (positions 512 r + tid) into the data VGPRs; lanes past `bytes` read 0 (buffer range)
__device__ __forceinline__ void vload(const double* src, uint32_t bytes, int tid) {
    const uint64_t a = (uint64_t)src;
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    u32x4 rs;
    rs.x = __builtin_amdgcn_readfirstlane((uint32_t)a);
    rs.y = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32) & 0xFFFFu);
    rs.z = __builtin_amdgcn_readfirstlane(bytes);
    rs.w = 0x00020000u;  // raw buffer, gfx9 data format (ck.hpp CK_BUFFER_RESOURCE_3RD_DWORD)
    // the whole offset in the VGPR (the buffer range check ignores soffset): lanes past `bytes` read 0
    const uint32_t vo = (uint32_t)tid * 8u;
    uint32_t vt;
    asm volatile(SVO_VROWS_ASM "s_waitcnt vmcnt(0)"
                 : [vt] "=&v"(vt)
                 : [vo] "v"(vo), [rs] "s"(rs)
                 : "memory", "v80", "v81", "v82", "v83", "v84", "v85", "v86", "v87", "v88", "v89", "v90", "v91", "v92", "v93", "v94", "v95", "v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108", "v109", "v110", "v111", "v112", "v113", "v114", "v115", "v116", "v117", "v118", "v119", "v120", "v121", "v122", "v123", "v124", "v125", "v126", "v127", "v128", "v129", "v130", "v131", "v132", "v133", "v134", "v135", "v136", "v137", "v138", "v139", "v140", "v141", "v142", "v143", "v144", "v145", "v146", "v147", "v148", "v149", "v150", "v151", "v152", "v153", "v154", "v155", "v156", "v157", "v158", "v159", "v160", "v161", "v162", "v163", "v164", "v165", "v166", "v167", "v168", "v169", "v170", "v171", "v172", "v173", "v174", "v175", "v176", "v177", "v178", "v179", "v180", "v181", "v182", "v183", "v184", "v185", "v186", "v187", "v188", "v189", "v190", "v191", "v192", "v193", "v194", "v195", "v196", "v197", "v198", "v199", "v200", "v201", "v202", "v203", "v204", "v205", "v206", "v207", "v208", "v209", "v210", "v211", "v212", "v213", "v214", "v215", "v216", "v217", "v218", "v219", "v220", "v221", "v222", "v223", "v224", "v225", "v226", "v227", "v228", "v229", "v230", "v231", "v232", "v233", "v234", "v235", "v236", "v237", "v238", "v239", "v240", "v241", "v242", "v243", "v244", "v245", "v246", "v247", "v248", "v249", "v250", "v251", "v252", "v253", "v254", "v255");
}

template <int R>
struct VSel {
    static_assert(R == 98, "register layout: rows 0..87 in v80..v255, 88..97 in LDS");
    static constexpr int kSteps = R * kVW;
    static constexpr int kKl = (kSteps + 63) / 64;  // scan entries per lane
    VShared<R>& sh;
    double* gseg;        // the pair's global scratch: the heap select's segment (depth limit only)
    uint32_t gdummy;     // its per-lane dummy slots (gseg[gdummy + lane], past every position)
    VDiag* dg;           // diagnostics (debug kernel) or nullptr
    uint32_t M, nth;
    int tid, lane, wave;
    // block-uniform selection state
    uint32_t f, l;
    int depth;
    bool rec;
    double lo_val;
    int P;
    bool small_round = false;  // (stamps build: the current block round has < 2048 positions)

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
        for (int r = rlo > kVRegRows ? rlo : kVRegRows; r <= rhi; ++r) {
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
        vload(src, M * 8u, tid);  // (rows past M hold 0: never inside a segment)
        for (int r = kVRegRows; r < R; ++r) {
            const uint32_t q = (uint32_t)r * kVT + (uint32_t)tid;
            sh.lrow[r - kVRegRows][tid] = q < M ? src[q] : 0.0;
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
        asm volatile(SVO_VLDS_ASM "s_waitcnt lgkmcnt(0)"
                     :
                     : [a] "v"(a)
                     : "memory", "v80", "v81", "v82", "v83", "v84", "v85", "v86", "v87", "v88", "v89", "v90", "v91", "v92", "v93", "v94", "v95", "v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108", "v109", "v110", "v111", "v112", "v113", "v114", "v115", "v116", "v117", "v118", "v119", "v120", "v121", "v122", "v123", "v124", "v125", "v126", "v127", "v128", "v129", "v130", "v131", "v132", "v133", "v134", "v135", "v136", "v137", "v138", "v139", "v140", "v141", "v142", "v143", "v144", "v145", "v146", "v147", "v148", "v149", "v150", "v151", "v152", "v153", "v154", "v155", "v156", "v157", "v158", "v159", "v160", "v161", "v162", "v163", "v164", "v165", "v166", "v167", "v168", "v169", "v170", "v171", "v172", "v173", "v174", "v175", "v176", "v177", "v178", "v179", "v180", "v181", "v182", "v183", "v184", "v185", "v186", "v187", "v188", "v189", "v190", "v191", "v192", "v193", "v194", "v195", "v196", "v197", "v198", "v199", "v200", "v201", "v202", "v203", "v204", "v205", "v206", "v207", "v208", "v209", "v210", "v211", "v212", "v213", "v214", "v215", "v216", "v217", "v218", "v219", "v220", "v221", "v222", "v223", "v224", "v225", "v226", "v227", "v228", "v229", "v230", "v231", "v232", "v233", "v234", "v235", "v236", "v237", "v238", "v239", "v240", "v241", "v242", "v243", "v244", "v245", "v246", "v247", "v248", "v249", "v250", "v251", "v252", "v253", "v254", "v255");
    }
    // preloaded: the rows were loaded already (the MAD pass's rows, during the median pass's one-wave rounds)
    __device__ __forceinline__ void load(const double* src, bool mad, double med, bool preloaded) {
        if (!preloaded) load_raw(src);
        if (mad) {  // src/algorithm.cpp:860-863 (DBL_MAX stays DBL_MAX)
            const uint64_t mb = uni(__builtin_bit_cast(uint64_t, med));
            asm volatile(SVO_VMAD_ASM ::[m] "s"(mb)
                         : "v80", "v81", "v82", "v83", "v84", "v85", "v86", "v87", "v88", "v89", "v90", "v91", "v92", "v93", "v94", "v95", "v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108", "v109", "v110", "v111", "v112", "v113", "v114", "v115", "v116", "v117", "v118", "v119", "v120", "v121", "v122", "v123", "v124", "v125", "v126", "v127", "v128", "v129", "v130", "v131", "v132", "v133", "v134", "v135", "v136", "v137", "v138", "v139", "v140", "v141", "v142", "v143", "v144", "v145", "v146", "v147", "v148", "v149", "v150", "v151", "v152", "v153", "v154", "v155", "v156", "v157", "v158", "v159", "v160", "v161", "v162", "v163", "v164", "v165", "v166", "v167", "v168", "v169", "v170", "v171", "v172", "v173", "v174", "v175", "v176", "v177", "v178", "v179", "v180", "v181", "v182", "v183", "v184", "v185", "v186", "v187", "v188", "v189", "v190", "v191", "v192", "v193", "v194", "v195", "v196", "v197", "v198", "v199", "v200", "v201", "v202", "v203", "v204", "v205", "v206", "v207", "v208", "v209", "v210", "v211", "v212", "v213", "v214", "v215", "v216", "v217", "v218", "v219", "v220", "v221", "v222", "v223", "v224", "v225", "v226", "v227", "v228", "v229", "v230", "v231", "v232", "v233", "v234", "v235", "v236", "v237", "v238", "v239", "v240", "v241", "v242", "v243", "v244", "v245", "v246", "v247", "v248", "v249", "v250", "v251", "v252", "v253", "v254", "v255");
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
    // candidate q of the next round (slot i): its owner publishes the pre-value and, if q is one of this round's
    // swap targets (side: 0 GE ranked from the left, 1 LE ranked from the right, rank <= ks), its rank, from the
    // step's record (masked to the round's segment at the classification) and the step's prefix (written by
    // this same wave in the scan)
    __device__ __forceinline__ void publish_cand(uint32_t q, int i, uint32_t ks, int side, uint32_t totL) {
        if (((q >> 6) & (kVW - 1)) != (uint32_t)wave) return;
        const double x = row_val((int)(q >> 9));
        uint32_t k = 0;
        if (ks) {
            const uint32_t s = q >> 6, b = q & 63u;
            const uint4 m4 = sh.rec[s];
            const uint64_t m = side ? ((uint64_t)uni(m4.w) << 32) | uni(m4.z) : ((uint64_t)uni(m4.y) << 32) | uni(m4.x);
            if ((m >> b) & 1ull) {
                const uint32_t pp = uni(sh.pre[s]);
                const uint32_t below = popc(m & low_mask(b));
                k = side ? totL - ((pp >> 16) + below) : (pp & 0xFFFFu) + below + 1u;
                if (k > ks) k = 0;
            }
        }
        if ((uint32_t)lane == (q & 63u)) {
            sh.pub[i] = x;
            sh.pubk[i] = k;
        }
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
    // This wave's rows of [f, l): only the first and the last can be partial; the first also drops position
    // f (the pivot) from GE.  Interior rows take full masks without any per-row mask arithmetic.
    struct WaveRows {
        int rlo, rhi;
        uint64_t ge_first, le_first, last;
        __device__ __forceinline__ uint64_t ge(int r) const { return r == rlo ? ge_first : (r == rhi ? last : ~0ull); }
        __device__ __forceinline__ uint64_t le(int r) const { return r == rlo ? le_first : (r == rhi ? last : ~0ull); }
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
    __device__ __forceinline__ void classify(double p, uint32_t ch, double x0) {
        // std::iter_swap(first, chosen) of __move_median_to_first, in the owners' registers
        if (((f >> 6) & (kVW - 1)) == (uint32_t)wave) row_set((int)(f >> 9), f & 63u, p);
        if (((ch >> 6) & (kVW - 1)) == (uint32_t)wave) row_set((int)(ch >> 9), ch & 63u, x0);
        const WaveRows w = wave_segment(f >> 6, (l - 1) >> 6);
        if (w.rlo > w.rhi) return;
        uint4* const recw = sh.rec + wave;
        auto put = [&](int r, uint64_t ge, uint64_t le) __attribute__((always_inline)) {
            if (lane == 0) recw[r * kVW] = make_uint4((uint32_t)ge, (uint32_t)(ge >> 32), (uint32_t)le, (uint32_t)(le >> 32));
        };
        // the wave's first and last rows can be partial (the first also drops position f from GE): masked
        // one at a time; the rows between take the full compare masks with no scalar mask arithmetic
        auto edge = [&](int r, uint64_t gm, uint64_t lm) __attribute__((always_inline)) {
            uint64_t ge, le;
            if (r < kVRegRows) {
                vcmp2(r, p, ge, le);
            } else {
                const double x = sh.lrow[r - kVRegRows][tid];
                ge = __ballot(!(x < p));
                le = __ballot(!(p < x));
            }
            put(r, ge & gm, le & lm);
        };
        edge(w.rlo, w.ge_first, w.le_first);
        if (w.rhi > w.rlo) edge(w.rhi, w.last, w.last);
        const int ra = w.rlo + 1, rb = w.rhi - 1;  // interior rows
        const int r1 = rb < kVRegRows - 1 ? rb : kVRegRows - 1;
        int r = ra;
        // LDS byte address of this wave's record of row 0 (row r: + r * 128)
        const uint32_t rec0 = (uint32_t)(uintptr_t)(recw);
        for (; r + 3 <= r1; r += 4) {
            uint64_t ge[4], le[4];
            vcmp2x4(r, p, ge, le);
            if (lane == 0) {
                const uint32_t ad = rec0 + (uint32_t)r * (uint32_t)(kVW * sizeof(uint4));
                rec_put<0>(ad, ge[0], le[0]);
                rec_put<kVW * 16>(ad, ge[1], le[1]);
                rec_put<2 * kVW * 16>(ad, ge[2], le[2]);
                rec_put<3 * kVW * 16>(ad, ge[3], le[3]);
            }
        }
        for (; r <= r1; ++r) {
            uint64_t ge, le;
            vcmp2(r, p, ge, le);
            put(r, ge, le);
        }
        for (int r = ra > kVRegRows ? ra : kVRegRows; r <= rb; ++r) {
            const double x = sh.lrow[r - kVRegRows][tid];
            put(r, __ballot(!(x < p)), __ballot(!(p < x)));
        }
    }

    // ------------------------------------------------------------------ 2. scan and searches (every wave)
    struct Scan {
        uint32_t pk[kKl];  // exclusive #GE | #LE << 16 before entry lane * K + i (i < K)
        uint32_t sf, E, K, totG, totL;  // K = ceil(E / 64) entries per lane: small segments scan 1-2
    };
    __device__ __forceinline__ void scan(Scan& S) {
        S.sf = f >> 6;
        S.E = ((l - 1) >> 6) - S.sf + 1;
        S.K = (S.E + 63u) >> 6;
        // #GE | #LE << 16 packed in one word (both <= 50 176: the low half never carries into the high one), so
        // one DPP scan serves both counts
        if (S.K == 1) {  // one entry per lane (segments of <= 4096 positions): no slot loops
            const uint32_t e = (uint32_t)lane;
            uint32_t c = 0;
            if (e < S.E) {
                const uint4 m = sh.rec[S.sf + e];
                c = ((uint32_t)__popc(m.x) + (uint32_t)__popc(m.y)) | (((uint32_t)__popc(m.z) + (uint32_t)__popc(m.w)) << 16);
            }
            const uint32_t it = wave_incl_scan(c);
            S.pk[0] = it - c;
            if (e < S.E && ((S.sf + e) & (kVW - 1)) == (uint32_t)wave) sh.pre[S.sf + e] = S.pk[0];
            const uint32_t tot = uni(lane_read(it, 63));
            S.totG = tot & 0xFFFFu;
            S.totL = tot >> 16;
            return;
        }
        uint32_t t = 0;
#pragma unroll
        for (int i = 0; i < kKl; ++i) {
            S.pk[i] = 0;
            if ((uint32_t)i < S.K) {
                const uint32_t e = (uint32_t)lane * S.K + (uint32_t)i;
                uint32_t c = 0;
                if (e < S.E) {
                    const uint4 m = sh.rec[S.sf + e];
                    c = ((uint32_t)__popc(m.x) + (uint32_t)__popc(m.y)) | (((uint32_t)__popc(m.z) + (uint32_t)__popc(m.w)) << 16);
                }
                S.pk[i] = t;
                t += c;
                if ((i & (kScanGroup - 1)) == kScanGroup - 1) asm volatile("" ::: "memory");  // bounded reads in flight
            }
        }
        const uint32_t it = wave_incl_scan(t);
        const uint32_t off = it - t;
#pragma unroll
        for (int i = 0; i < kKl; ++i) {
            if ((uint32_t)i < S.K) {
                S.pk[i] += off;
                const uint32_t e = (uint32_t)lane * S.K + (uint32_t)i;
                if (e < S.E && ((S.sf + e) & (kVW - 1)) == (uint32_t)wave) sh.pre[S.sf + e] = S.pk[i];
            }
        }
        const uint32_t tot = uni(lane_read(it, 63));
        S.totG = tot & 0xFFFFu;
        S.totL = tot >> 16;
    }
    // the packed prefix of a block-uniform entry
    __device__ __forceinline__ uint32_t pk_at(const Scan& S, uint32_t e) const {
        const uint32_t li = uni(e / S.K), ii = uni(e - li * S.K);
        // an and-or chain in asm (one v_and_or_b32 per slot): written as plain selects, the compiler turned it
        // into an indexed load and kept pk[] in scratch memory (a store per entry every scan, a memory round
        // trip per lookup)
        if (S.K == 1) return uni(lane_read(S.pk[0], (int)e));  // (one entry per lane: most rounds)
        uint32_t x = 0;
#pragma unroll
        for (int i = 0; i < kKl; ++i) {
            const uint32_t msk = ii == (uint32_t)i ? ~0u : 0u;
            asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(x) : "v"(S.pk[i]), "s"(msk), "v"(x));
        }
        return uni(lane_read(x, (int)li));
    }
    __device__ __forceinline__ uint64_t rec_mask(uint32_t s, int kind) const {
        const uint4 m = sh.rec[s];
        return kind ? ((uint64_t)uni(m.w) << 32) | uni(m.z) : ((uint64_t)uni(m.y) << 32) | uni(m.x);
    }
    // the rank-th (1-based) GE (kind 0) or LE (kind 1) position from the left; cnt = #entries whose prefix is
    // below the rank (so the entry cnt - 1 holds it)
    __device__ __forceinline__ uint32_t locate(const Scan& S, uint32_t cnt, int kind, uint32_t rank) const {
        const uint32_t e = cnt - 1u;
        const uint32_t pk = pk_at(S, e);
        const uint32_t pre = kind ? pk >> 16 : pk & 0xFFFFu;
        return (S.sf + e) * 64u + wave_select_bit(rec_mask(S.sf + e, kind), rank - pre - 1u);
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
    // ------------------------------------------------------------------ 3. the exchange
    // side 0: GE positions ranked from the left (L_k), side 1: LE positions ranked from the right (R_k), over
    // the steps [s0, s1]; ranks k in (k0, k1]: kWrite stores the value in mb[k - 1 - k0], else the position
    // takes it.  The masks are recomputed from the registers (the same compares as the classification).
    // chunked (more than one exchange chunk): the masks come from the records instead, since an earlier
    // chunk's targets may have changed registers the recompute would read (the round then ends with a barrier,
    // so no wave reads the records while a faster one classifies the next round)
    // this wave's step prefixes, lane j: row j (pre0) and row 64 + j (pre1), read once per round for both
    // exchange phases
    __device__ __forceinline__ void wave_prefixes(uint32_t& pre0, uint32_t& pre1) const {
        pre0 = sh.pre[((uint32_t)lane * kVW + (uint32_t)wave) % kSteps];
        pre1 = sh.pre[(((uint32_t)lane + 64u) * kVW + (uint32_t)wave) % kSteps];
    }
    template <bool kWrite>
    __device__ __forceinline__ void exchange(int side, uint32_t s0, uint32_t s1, double p, uint32_t totL, uint32_t k0,
                                             uint32_t k1, bool chunked, uint32_t pre0, uint32_t pre1) {
        const WaveRows w = wave_segment(s0, s1);
        if (w.rlo > w.rhi) return;
        // a lane's mailbox index: ranks k0 < k <= k1 of m (okm) use mbx[k - 1 - k0], the other lanes their
        // dummy slot mbx[kMbCap + lane].  kk = k - 1 - k0 is one mbcnt over a scalar base (side 0: ranks from
        // the left, pp's GE count + the GE lanes below + 1; side 1: ranks from the right, totL - (pp's LE
        // count + the LE lanes below)); the range test is one unsigned compare, the slot one v_cndmask on
        // the SGPR mask
        const uint32_t nk = k1 - k0;
        const uint32_t dslot = kMbCap + (uint32_t)lane;
        // the scalar part of kk for the step prefix pp (an opaque copy: the compiler would otherwise fold the
        // side-1 base back into the per-lane arithmetic)
        auto kbase = [&](uint32_t pp) __attribute__((always_inline)) -> uint32_t {
            uint32_t b = side == 0 ? (pp & 0xFFFFu) - k0 : totL - 1u - k0 - (pp >> 16);
            asm volatile("" : "+s"(b));
            return b;
        };
        auto slot_pp = [&](uint32_t pp, uint64_t m, uint64_t& okm) __attribute__((always_inline)) -> uint32_t {
            const uint32_t b = kbase(pp);
            const uint32_t kk = side == 0 ? __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, b))
                                          : b - lanes_below(m);
            okm = m & __ballot(kk < nk);
            return lane_sel(okm, kk, dslot);
        };
        auto slot = [&](int r, uint64_t m, uint64_t& okm) __attribute__((always_inline)) -> uint32_t {
            return slot_pp(r < 64 ? lane_read(pre0, r) : lane_read(pre1, r - 64), m, okm);
        };
        // the side's mask of row r (register row, or the LDS row value x); the records when chunked (masked
        // at the classification); interior rows need no range mask (the edge rows are peeled below)
        auto mask = [&](int r, double x, bool reg) __attribute__((always_inline)) -> uint64_t {
            if (chunked) return rec_mask((uint32_t)(r * kVW + wave), side);
            if (side == 0) return reg ? vcmp_ge(r, p) : __ballot(!(x < p));
            return reg ? vcmp_le(r, p) : __ballot(!(p < x));
        };
        double* const mbx = sh.mbx;
        // register rows, four per iteration (independent chains: their compares, ranks and LDS accesses
        // overlap), then the rest one at a time; rows below 64 take their prefixes from pre0, the others from
        // pre1 (two loops: one readlane per row, no select)
        auto reg_rows = [&](int ra, int rb, uint32_t prex, int roff) __attribute__((always_inline)) {
            int r = ra;
            for (; r + 3 <= rb; r += 4) {
                uint64_t m[4];
                if (chunked) {
#pragma unroll
                    for (int j = 0; j < 4; ++j) m[j] = rec_mask((uint32_t)((r + j) * kVW + wave), side);
                } else {
                    if (side == 0) vcmpx4<0>(r, p, m);
                    else vcmpx4<1>(r, p, m);
                }
                uint64_t okm[4];
                uint32_t a[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) a[j] = slot_pp(lane_read(prex, r + j - roff), m[j], okm[j]);
                if (kWrite) {
                    double x[4];
                    vgetx4(r, x);
#pragma unroll
                    for (int j = 0; j < 4; ++j) mbx[a[j]] = x[j];
                } else {
                    double t[4];
#pragma unroll
                    for (int j = 0; j < 4; ++j) t[j] = mbx[a[j]];
                    vselx4(r, t, okm);
                }
            }
            for (; r <= rb; ++r) {
                uint64_t okm;
                const uint32_t a0 = slot_pp(lane_read(prex, r - roff), mask(r, 0.0, true), okm);
                if (kWrite) {
                    mbx[a0] = vget(r);
                } else {
                    const double t0 = mbx[a0];
                    vsel(r, t0, okm);
                }
            }
        };
        // one row with an explicit range mask gm (register or LDS row)
        auto one_row = [&](int r, uint64_t gm) __attribute__((always_inline)) {
            uint64_t okm;
            if (r < kVRegRows) {
                const uint32_t a0 = slot(r, mask(r, 0.0, true) & gm, okm);
                if (kWrite) {
                    mbx[a0] = vget(r);
                } else {
                    const double t0 = mbx[a0];
                    vsel(r, t0, okm);
                }
            } else {
                double& y = sh.lrow[r - kVRegRows][tid];
                const double x = y;
                const uint32_t a = slot(r, mask(r, x, false) & gm, okm);
                if (kWrite) {
                    mbx[a] = x;
                } else {
                    const double t = mbx[a];
                    y = ((okm >> lane) & 1ull) ? t : x;
                }
            }
        };
        // edge rows (partial: masked), then the interior rows (full masks)
        one_row(w.rlo, side == 0 ? w.ge_first : w.le_first);
        if (w.rhi > w.rlo) one_row(w.rhi, w.last);
        const int ra = w.rlo + 1, rb = w.rhi - 1;
        const int r1i = rb < kVRegRows - 1 ? rb : kVRegRows - 1;
        reg_rows(ra, r1i < 63 ? r1i : 63, pre0, 0);
        reg_rows(ra > 64 ? ra : 64, r1i, pre1, 64);
        for (int r = ra > kVRegRows ? ra : kVRegRows; r <= rb; ++r) one_row(r, ~0ull);
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
        Scan S;
        scan(S);
        VSTAMP(8);
        const uint32_t totL = S.totL, totG = S.totG;
        // the crossing: the last entry whose start has G < Lc (entry 0 always: G = 0 < Lc = totL)
        uint32_t c = 0, es;
        if (S.K == 1) {  // one entry per lane: a ballot counts them
            es = popc(__ballot((uint32_t)lane < S.E && (S.pk[0] & 0xFFFFu) < totL - (S.pk[0] >> 16))) - 1u;
        } else {
#pragma unroll
            for (int i = 0; i < kKl; ++i) {
                const uint32_t e = (uint32_t)lane * S.K + (uint32_t)i;
                if ((uint32_t)i < S.K && e < S.E) c += (S.pk[i] & 0xFFFFu) < totL - (S.pk[i] >> 16) ? 1u : 0u;
            }
            es = uni(wave_sum_u(c)) - 1u;
        }
        const uint32_t pke = pk_at(S, es);
        const uint4 me4 = sh.rec[S.sf + es];  // (both masks of the crossing entry in one read)
        const uint64_t mge = ((uint64_t)uni(me4.y) << 32) | uni(me4.x), mle = ((uint64_t)uni(me4.w) << 32) | uni(me4.z);
        const uint32_t ks = uni(wave_crossing_ks(pke & 0xFFFFu, totL - (pke >> 16), mge, mle));
        VSTAMP(9);
        // L_{Ks+1} (GE rank Ks + 1), R_{Ks} (LE rank totL - Ks + 1 from the left), L_{Ks}.  All three sit next to
        // the crossing split, so they are looked for in the crossing entry first (its prefix and masks are at
        // hand); only if one of them lies in another entry do the ranks take the full search (a packed count
        // over every entry, then a lookup and a bit select per rank).
        const uint32_t ra = ks + 1u, rb = totL - ks + 1u, rc = ks;
        const uint32_t G0 = pke & 0xFFFFu, L0 = pke >> 16, cg = popc(mge), cl = popc(mle);
        const uint32_t ebase = (S.sf + es) * 64u;
        const bool in_a = ra > totG || (ra > G0 && ra <= G0 + cg);
        const bool in_b = ks == 0 || (rb > L0 && rb <= L0 + cl);
        const bool in_c = ks == 0 || (rc > G0 && rc <= G0 + cg);
        uint32_t cs = 0;  // the packed count of every entry below each rank, only when a rank lies elsewhere
        if (!(in_a && in_b && in_c)) {
            c = 0;
#pragma unroll
            for (int i = 0; i < kKl; ++i) {
                const uint32_t e = (uint32_t)lane * S.K + (uint32_t)i;
                if ((uint32_t)i < S.K && e < S.E) {
                    const uint32_t pg = S.pk[i] & 0xFFFFu, pl = S.pk[i] >> 16;
                    c += (pg < ra ? 1u : 0u) + (pl < rb ? 1u << 10 : 0u) + (pg < rc ? 1u << 20 : 0u);
                }
            }
            cs = uni(wave_sum_u(c));
        }
        const uint32_t lk1 = ra > totG ? kNone
                             : in_a ? ebase + uni(wave_select_bit(mge, ra - G0 - 1u)) : uni(locate(S, cs & 1023u, 0, ra));
        const uint32_t rk = ks == 0 ? kNone
                            : in_b ? ebase + uni(wave_select_bit(mle, rb - L0 - 1u)) : uni(locate(S, (cs >> 10) & 1023u, 1, rb));
        const uint32_t lk = ks == 0 ? kNone
                            : in_c ? ebase + uni(wave_select_bit(mge, rc - G0 - 1u)) : uni(locate(S, cs >> 20, 0, rc));
        const uint32_t cut = lk1 < rk ? lk1 : rk;
        VSTAMP(10);
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
        // the next round's candidates: each owner publishes its pre-value and its target rank (the mailbox
        // slot that will hold its new value), from its own step's prefix and record; the other waves do nothing
        if (need) {
#pragma unroll
            for (int i = 0; i < 4; ++i) publish_cand(cq[i], i, ks, tgt_side, totL);
        }
        const uint32_t sl = (l - 1) >> 6;
        const uint32_t s0L = S.sf, s1L = lk != kNone ? lk >> 6 : 0u;           // L_k, k <= Ks
        const uint32_t s0R = rk != kNone ? rk >> 6 : sl + 1u, s1R = sl;       // R_k, k <= Ks
        // Ks beyond the mailbox: chunks of kMbCap ranks, the masks from the records (see exchange).
        const uint32_t nch = ks == 0 ? 1u : (ks + kMbCap - 1u) / kMbCap;
        uint32_t ck[4] = {0, 0, 0, 0};  // the candidates' target ranks (0: not a target)
        uint32_t pre0 = 0, pre1 = 0;
        if (ks) wave_prefixes(pre0, pre1);
        VSTAMP(3);
        for (uint32_t it = 0; it < nch; ++it) {
            const uint32_t ci = it;
            const uint32_t k0 = ci * kMbCap, k1 = ks < k0 + kMbCap ? ks : k0 + kMbCap;
            if (ks) {
                if (src_side == 0) exchange<true>(0, s0L, s1L, p, totL, k0, k1, nch > 1, pre0, pre1);
                else exchange<true>(1, s0R, s1R, p, totL, k0, k1, nch > 1, pre0, pre1);
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
                if (tgt_side == 0) exchange<false>(0, s0L, s1L, p, totL, k0, k1, nch > 1, pre0, pre1);
                else exchange<false>(1, s0R, s1R, p, totL, k0, k1, nch > 1, pre0, pre1);
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
#if defined(SVO_STAMPS)
        if (dg && tid == 0 && dg->nlog < 64) {
            dg->log[dg->nlog][0] = S0;
            dg->log[dg->nlog][1] = (uint32_t)(clock64() - tround);
            ++dg->nlog;
        }
#endif
        f = nf;
        l = nl;
    }

    // ------------------------------------------------------------------ rounds of <= 512 positions (wave 0)
    // No barriers: wave 0 takes the segment (seg[i] = position f0 + i, from the dump) into its data rows 0..7
    // (position f0 + 64 j + L in lane L of row j; the rows' own values are dead after the dump), so a round
    // reads no segment memory: the candidates are readlanes, the masks compares, the counts / crossing / rank
    // searches scalars and ballots, the swaps go through the mailbox mb (a wave's LDS accesses complete in
    // program order) into the rows by masked selects.  Stops at <= 3 positions or depth 0; then the rows go
    // back to seg for the final sort or the heap select.
    __device__ __forceinline__ double cand_at(uint32_t q) const {
        return uni(lane_read(vget((int)(q >> 6)), (int)(q & 63u)));
    }
    __device__ __forceinline__ void wave_rounds(double* seg, double* mb, uint32_t& nrounds) {
        const uint32_t f0 = f, me = (uint32_t)lane;
        uint32_t fr = 0, lr = l - f;
        const uint32_t nrel = nth - f0;
#pragma unroll
        for (int j = 0; j < (int)(kOneWave / 64); ++j) vset(j, seg[64 * j + lane]);
        // the mailbox and each lane's dummy slot as indices into sh.mbx
        const uint32_t mb0 = (uint32_t)(mb - sh.mbx), dslot = kMbCap + me;
        double* const mbx = sh.mbx;
        // per-step data of a round in VGPR lanes (lane j = step j): the GE / LE masks and the #GE / #LE before
        // the step; the loops run over the live steps js..je only and the searches are ballots over the lanes
        while (lr - fr > 3 && depth > 0) {
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
            const uint32_t js = fr >> 6, je = (lr - 1) >> 6;
            uint32_t gel = 0, geh = 0, lel = 0, leh = 0, pkv = 0;  // lane j: step j's masks, packed #GE | #LE << 16 before it
            uint32_t tG = 0, tL = 0;
            for (uint32_t j = js; j <= je; ++j) {
                uint64_t ge, le;
                vcmp2((int)j, pe, ge, le);
                const uint32_t base = 64u * j;
                const uint32_t lo = fr > base ? fr - base : 0u;
                const uint32_t hi = lr - base < 64u ? lr - base : 64u;
                const uint64_t inm = low_mask(hi) & ~low_mask(lo);
                const uint64_t fb = js == j ? 1ull << (fr & 63u) : 0ull;
                ge &= inm & ~fb;
                le &= inm;
                gel = lane_put(gel, (uint32_t)ge, j, me);
                geh = lane_put(geh, (uint32_t)(ge >> 32), j, me);
                lel = lane_put(lel, (uint32_t)le, j, me);
                leh = lane_put(leh, (uint32_t)(le >> 32), j, me);
                pkv = lane_put(pkv, tG | (tL << 16), j, me);
                tG += popc(ge);
                tL += popc(le);
            }
            const bool live = me >= js && me <= je;
            const uint32_t gpl = pkv & 0xFFFFu, lpl = pkv >> 16;
            auto masks = [&](uint32_t j, uint64_t& ge, uint64_t& le) __attribute__((always_inline)) {
                ge = ((uint64_t)lane_read(geh, (int)j) << 32) | lane_read(gel, (int)j);
                le = ((uint64_t)lane_read(leh, (int)j) << 32) | lane_read(lel, (int)j);
            };
            // crossing: the last live step whose start has G < Lc (step js: G = 0 < Lc)
            const uint64_t cq = __ballot(live && gpl < tL - lpl);
            const uint32_t jc = 63u - (uint32_t)__builtin_clzll(cq);
            uint64_t a0, b0m;
            masks(jc, a0, b0m);
            const uint32_t pkc = lane_read(pkv, (int)jc);
            const uint32_t ks = uni(wave_crossing_ks(pkc & 0xFFFFu, tL - (pkc >> 16), a0, b0m));
            // the rank-th GE (kind 0) / LE (kind 1) position: the last live step starting below the rank
            auto rank_pos = [&](int kind, uint32_t rank) __attribute__((always_inline)) -> uint32_t {
                if (rank == 0 || rank > (kind ? tL : tG)) return kNone;
                const uint64_t q = __ballot(live && (kind ? lpl : gpl) < rank);
                const uint32_t jj = 63u - (uint32_t)__builtin_clzll(q);
                const uint32_t pp = lane_read(pkv, (int)jj);
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
            // sources to the mailbox, then the kept side's targets take it (masked selects into the rows)
            if (ks) {
                for (uint32_t j = js; j <= je; ++j) {
                    uint64_t ge, le;
                    masks(j, ge, le);
                    const uint64_t m = right ? ge : le;
                    const uint32_t pp = lane_read(pkv, (int)j);
                    const uint32_t k = right ? (pp & 0xFFFFu) + lanes_below(m) + 1u : tL - ((pp >> 16) + lanes_below(m));
                    const uint64_t okm = m & __ballot(k <= ks);
                    mbx[lane_sel(okm, mb0 + k - 1u, dslot)] = vget((int)j);
                }
                for (uint32_t j = js; j <= je; ++j) {
                    uint64_t ge, le;
                    masks(j, ge, le);
                    const uint64_t m = right ? le : ge;
                    const uint32_t pp = lane_read(pkv, (int)j);
                    const uint32_t k = right ? tL - ((pp >> 16) + lanes_below(m)) : (pp & 0xFFFFu) + lanes_below(m) + 1u;
                    const uint64_t okm = m & __ballot(k <= ks);
                    const double t = mbx[lane_sel(okm, mb0 + k - 1u, dslot)];
                    vsel((int)j, t, okm);
                }
            }
            if (right) fr = cut;
            else lr = cut;
        }
#pragma unroll
        for (int j = 0; j < (int)(kOneWave / 64); ++j) seg[64 * j + lane] = vget(j);
        f = f0 + fr;
        l = f0 + lr;
    }

    // ------------------------------------------------------------------ std::nth_element(vec, vec + nth)
    // (vec[nth - 1], vec[nth]) of the post-state, on thread 0
    // preload_next: load the raw rows for the MAD pass while wave 0 runs this pass's one-wave rounds (the other
    // waves' registers are free after the dump); returns through `preloaded` whether it did
    __device__ __forceinline__ void select(const double* src, bool mad, double med, bool preloaded, bool preload_next,
                                           double& hi, double& lo, bool& did_preload) {
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
        if (dg && tid == 0) {
            dg->nblock[P] = nblock;
            dg->cyc[P] = clock64() - t0;
        }
    }
};

// computeMedian / computeMAD (src/algorithm.cpp:834-865) with the reference's post-state; every thread
// returns med and mad.  M slots, n visible.
template <int R>
__device__ __forceinline__ void refv_robust_scale(const double* src, VShared<R>& sh, double* gseg, VDiag* dg, uint32_t M,
                                                  uint32_t n, double& med, double& mad) {
    VSel<R> s{sh, gseg, (uint32_t)((M + 63u) / 64u * 64u), dg};
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
        bool did = false;
        s.select(src, P == 1, m0, pre, P == 0, hi, lo, did);
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

template <int R>
__device__ __forceinline__ void scale_refv_pair(const AlignArgs& a, VShared<R>& sh) {
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
        refv_robust_scale<R>(a.scratch + (int64_t)pair * a.key_stride, sh,
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

// K2V: one 512-thread workgroup per pair, one pair per CU (all of its registers and 144 KB of LDS).
__global__ void __launch_bounds__(kVT, 1) 
align_scale_refv_kernel(AlignArgs a, int level) {
    __shared__ VShared<kVRows> sh;
    (void)level;
    scale_refv_pair<kVRows>(a, sh);
}

// svo_debug_robust_scale: the same selection on an arbitrary vector (one workgroup); out[0..1] med / mad,
// out[2..] diagnostics (rounds, chunked rounds, heap selects, cycles per pass)
__global__ void __launch_bounds__(kVT, 1) 
debug_robust_scale_v_kernel(const double* v, uint32_t M, uint32_t n, double* gseg, double* out) {
    __shared__ VShared<kVRows> sh;
    __shared__ VDiag dg;
    if (threadIdx.x == 0) dg = VDiag{};
    __syncthreads();
    double med = 0.0, mad = 0.0;
    refv_robust_scale<kVRows>(v, sh, gseg, &dg, M, n, med, mad);
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
        for (int i = 0; i < 128; ++i) out[24 + i] = i / 2 < (int)dg.nlog ? (double)dg.log[i / 2][i % 2] : -1.0;

    }
}

int64_t refv_max_slots() { return kVCap; }
void launch_scale_refv(const AlignArgs& a, int level, hipStream_t s) {
    hipLaunchKernelGGL(align_scale_refv_kernel, dim3(a.n_pairs), dim3(kVT), 0, s, a, level);
}
void launch_debug_robust_scale_v(const double* v, uint32_t M, uint32_t n, double* gseg, double* out, hipStream_t s) {
    hipLaunchKernelGGL(debug_robust_scale_v_kernel, dim3(1), dim3(kVT), 0, s, v, M, n, gseg, out);
}

}  // namespace svo
