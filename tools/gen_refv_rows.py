"""Generates semi-direct-visual-odometry_amd/csrc/refv_rows.h: K2V's asm on its fixed data registers.

K2V (csrc/align_refv.hip) keeps the residual vector of one pair in the VGPRs of one CU: row r < kRegRows of
every lane in the pair v[B + 2r : B + 2r + 1] above a register fence B (the compiler's own values stay below
it), the remaining rows in LDS.  Three layouts, one struct each:

  RowsA  B = 80, 88 register rows   (K2V's 98-row layout: vectors of <= 50 176 slots, the config-2 shape)
  RowsB  B = 72, 92 register rows   (the 118-row layout: <= 60 416 slots, frames of up to 2416 features at patch 5)
  RowsC  B = 64, 96 register rows   (the 128-row layout: <= 65 536 slots, frames of up to 2621 features at patch 5)

Every struct holds
  load(src, bytes, tid) / mad(med) / unstage(a)   the rows' buffer loads, the MAD pass's |x - med| in place, and
                                      wave 0's staged rows from LDS (one asm block each, every row named)
  vget / vset / vcmp2 / vcmp_ge / vcmp_le / vsel(r, ...)   a runtime row in VGPR indexing mode (base register B)
  cls4<Q>(p, acc[4])                  rows 4Q..4Q+3: the compares ge = !(x < p), le = !(p < x), each mask
                                      written to lane r & 63 of the row group's four accumulators (via VCC: the
                                      asm operand syntax cannot name one half of a compiler-chosen SGPR pair)

The asm blocks carry their own wait states (hipcc pads none inside a block): a VALU write of VCC read as a constant
by the next VALU needs one (cls4 orders its compares for it), a VALU write of a VGPR read by v_readlane needs one
(w1src / w1tgt open with s_nop 0; the exchange quads' readlanes come after four compares), and a VALU write of an
SGPR read by a buffer load needs five (load opens with s_nop 4: its descriptor may come straight from
v_readfirstlane).
  src4<Q, S>(p, pb) / src4e<Q, S>(p, pb, ra, len)   the sources of an exchange write the mailbox   (side S)
  tgt4<Q, S>(p, pb) / tgt4e<Q, S>(p, pb, ra, len)   the targets take the mailbox values            (side S)
                                      (the e forms test each row against the row range [ra, ra + len])
  w1src / w1tgt<Q, S>(ml, mh, pre, ks, tl1, mb)   rows 4Q..4Q+3 (< 32) of a one-wave round's exchange (wave 0,
                                      the segment in its rows 0 .. OW / 64 - 1): sources / targets
  fence()                             the marker `;@vfence B` the build check reads in each kernel

Every per-row decision of the quads happens inside the asm block, so the compiler has nothing to hoist across
quads (left to it, the row masks and slot bases of all quads were computed up front and spilled).  Side 0 ranks GE
positions from the left (mailbox slot k - 1 = #GE before the step + GE lanes below), side 1 ranks LE positions
from the right (slot = totL - 1 - #LE before the step - LE lanes below); pb holds the mailbox byte address of
each row's slot 0 (lane r & 63).  The lanes that take part are selected by EXEC (set from the row's mask, restored
once per block): no dummy slots, no value selects.  Every instruction counts: a wave issues at most one per four
cycles.

Every instruction that names a fixed data register carries a `;@vfix i[,j]` tag listing those operand positions:
tools/check_vreg_fence.py exempts exactly those operands from the kernel's fence and requires every other operand
below it.

usage: python3 tools/gen_refv_rows.py [out]  (writes the header; the output is committed, and
       tests/test_asm_checks.py regenerates it and fails on any difference)
"""
import os

LAYOUTS = (("RowsA", 80), ("RowsB", 72), ("RowsC", 64))
# the one-wave rounds' quads (rows 0 .. 4 W1QUADS - 1 of wave 0: one-wave segments of up to 256 W1QUADS positions)
W1QUADS = int(os.environ.get("SVO_GEN_W1QUADS", "8"))
# the quads' instruction-level parallelism form (cls4_ilp / exch_ilp): compares first, then independent per-row chains
ILP = os.environ.get("SVO_GEN_ILP", "1") == "1"
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "semi-direct-visual-odometry_amd",
                   "csrc", "refv_rows.h")


def asm(lines):
    return "\\n\\t".join(lines)


class Gen:
    def __init__(self, name, base):
        self.name, self.base = name, base
        self.rows = (256 - base) // 2
        assert self.rows % 4 == 0, "register rows come in quads"
        self.clob = ", ".join(f'"v{i}"' for i in range(base, 256))

    def reg(self, r):
        return f"v[{self.base + 2 * r}:{self.base + 2 * r + 1}]"

    # ---------------------------------------------------------------- whole-vector blocks (inside the struct)
    def members(self):
        B, n = self.base, self.rows
        # s_nop 4 first: the descriptor's SGPRs may come straight from v_readfirstlane, and a VALU write of an SGPR
        # read by a VMEM instruction needs five wait states (hipcc pads none inside the block)
        load = ["s_nop 4"]
        for r in range(n):
            load += [f"v_add_u32 %[vt], 0x{r * 0x1000:x}, %[vo]",
                     f"buffer_load_dwordx2 {self.reg(r)}, %[vt], %[rs], 0 offen ;@vfix 0"]
        load.append("s_waitcnt vmcnt(0)")
        mad = []
        for r in range(n):
            mad += [f"v_add_f64 {self.reg(r)}, {self.reg(r)}, -%[m] ;@vfix 0,1",
                    f"v_and_b32 v{B + 2 * r + 1}, 0x7fffffff, v{B + 2 * r + 1} ;@vfix 0,2"]
        uns = [f"ds_read_b64 {self.reg(r)}, %[a] offset:{512 * r} ;@vfix 0" for r in range(n)] + ["s_waitcnt lgkmcnt(0)"]
        b0, b1 = f"v{B}", f"v{B + 1}"
        return f'''    static constexpr int kBase = {B};       // first data VGPR
    static constexpr int kRegRows = {n};    // rows in v{B}..v255
    static constexpr int kGenQuads = {n // 4};   // register quads with generated bodies (rows 0 .. {4 * (n // 4) - 1})
    static constexpr bool kTgt8 = {"true" if self.name == "RowsA" else "false"};  // tgt8: eight target rows per block
    static __device__ __forceinline__ void fence() {{ asm volatile(";@vfence {B}"); }}
    // rows 0..{n - 1} of src (positions 512 r + tid) into the data registers; lanes past `bytes` read 0 (buffer range)
    static __device__ __forceinline__ void load(const double* src, uint32_t bytes, int tid) {{
        const uint64_t a = (uint64_t)src;
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
        u32x4 rs;
        rs.x = __builtin_amdgcn_readfirstlane((uint32_t)a);
        rs.y = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32) & 0xFFFFu);
        rs.z = __builtin_amdgcn_readfirstlane(bytes);
        rs.w = 0x00020000u;  // raw buffer, gfx9 data format
        // the whole offset in the VGPR (the buffer range check ignores soffset): lanes past `bytes` read 0
        const uint32_t vo = (uint32_t)tid * 8u;
        uint32_t vt;
        asm volatile("{asm(load)}"
                     : [vt] "=&v"(vt)
                     : [vo] "v"(vo), [rs] "s"(rs)
                     : "memory", {self.clob});
    }}
    // the MAD pass's |x - med| on every register row in place (src/algorithm.cpp:860-863): one subtraction and one
    // sign clear per row (the same IEEE result as fabs(x - med))
    static __device__ __forceinline__ void mad(uint64_t m) {{
        asm volatile("{asm(mad)}" ::[m] "s"(m) : {self.clob});
    }}
    // wave 0's rows from their LDS staging (stg[64 r + lane]: byte offset 512 r from the lane's address a)
    static __device__ __forceinline__ void unstage(uint32_t a) {{
        asm volatile("{asm(uns)}" : : [a] "v"(a) : "memory", {self.clob});
    }}
    // the lane's value in block-uniform row r / store x there (VGPR indexing mode: M0 is written; the compiler's
    // code never uses M0 in these kernels, which the build check verifies)
    static __device__ __forceinline__ double vget(int r) {{
        uint32_t lo, hi;
        asm volatile("s_set_gpr_idx_on %2, gpr_idx(SRC0)\\n\\tv_mov_b32 %0, {b0} ;@vfix 1\\n\\tv_mov_b32 %1, {b1} ;@vfix 1\\n\\ts_set_gpr_idx_off"
                     : "=v"(lo), "=v"(hi)
                     : "s"(__builtin_amdgcn_readfirstlane(2 * r)));
        return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
    }}
    static __device__ __forceinline__ void vset(int r, double x) {{
        const uint64_t u = __builtin_bit_cast(uint64_t, x);
        asm volatile("s_set_gpr_idx_on %2, gpr_idx(DST)\\n\\tv_mov_b32 {b0}, %0 ;@vfix 0\\n\\tv_mov_b32 {b1}, %1 ;@vfix 0\\n\\ts_set_gpr_idx_off"
                     :
                     : "v"((uint32_t)u), "v"((uint32_t)(u >> 32)), "s"(__builtin_amdgcn_readfirstlane(2 * r)));
    }}
    // the row compares straight on the data registers: ge = !(x < p), le = !(p < x)
    static __device__ __forceinline__ void vcmp2(int r, double p, uint64_t& ge, uint64_t& le) {{
        asm volatile("s_set_gpr_idx_on %2, gpr_idx(SRC0)\\n\\tv_cmp_nlt_f64 %0, v[{B}:{B + 1}], %3 ;@vfix 1\\n\\tv_cmp_ngt_f64 %1, v[{B}:{B + 1}], %3 ;@vfix 1\\n\\ts_set_gpr_idx_off"
                     : "=&s"(ge), "=&s"(le)
                     : "s"(__builtin_amdgcn_readfirstlane(2 * r)), "s"(p));
    }}
    static __device__ __forceinline__ uint64_t vcmp_ge(int r, double p) {{
        uint64_t m;
        asm volatile("s_set_gpr_idx_on %1, gpr_idx(SRC0)\\n\\tv_cmp_nlt_f64 %0, v[{B}:{B + 1}], %2 ;@vfix 1\\n\\ts_set_gpr_idx_off"
                     : "=s"(m)
                     : "s"(__builtin_amdgcn_readfirstlane(2 * r)), "s"(p));
        return m;
    }}
    static __device__ __forceinline__ uint64_t vcmp_le(int r, double p) {{
        uint64_t m;
        asm volatile("s_set_gpr_idx_on %1, gpr_idx(SRC0)\\n\\tv_cmp_ngt_f64 %0, v[{B}:{B + 1}], %2 ;@vfix 1\\n\\ts_set_gpr_idx_off"
                     : "=s"(m)
                     : "s"(__builtin_amdgcn_readfirstlane(2 * r)), "s"(p));
        return m;
    }}
    // the lanes of m take x in row r (DST and SRC0 indexed: the register itself is the kept value)
    static __device__ __forceinline__ void vsel(int r, double x, uint64_t m) {{
        const uint64_t u = __builtin_bit_cast(uint64_t, x);
        asm volatile("s_set_gpr_idx_on %3, gpr_idx(SRC0,DST)\\n\\tv_cndmask_b32 {b0}, {b0}, %0, %2 ;@vfix 0,1\\n\\tv_cndmask_b32 {b1}, {b1}, %1, %2 ;@vfix 0,1\\n\\ts_set_gpr_idx_off"
                     :
                     : "v"((uint32_t)u), "v"((uint32_t)(u >> 32)), "s"(m), "s"(__builtin_amdgcn_readfirstlane(2 * r)));
    }}
    template <int Q> static __device__ __forceinline__ void cls4(double p, uint32_t (&acc)[4]);
    template <int Q, int S> static __device__ __forceinline__ void src4(double p, uint32_t pb);
    template <int Q, int S> static __device__ __forceinline__ void tgt4(double p, uint32_t pb);
    template <int O, int S> static __device__ __forceinline__ void tgt8(double p, uint32_t pb);
    template <int Q, int S> static __device__ __forceinline__ void src4e(double p, uint32_t pb, uint32_t ra, uint32_t len);
    template <int Q, int S> static __device__ __forceinline__ void tgt4e(double p, uint32_t pb, uint32_t ra, uint32_t len);
    template <int Q, int S> static __device__ __forceinline__ void w1src(uint32_t ml, uint32_t mh, uint32_t pre, uint32_t ks,
                                                                        uint32_t tl1, uint32_t mb);
    template <int Q, int S> static __device__ __forceinline__ void w1tgt(uint32_t ml, uint32_t mh, uint32_t pre, uint32_t ks,
                                                                        uint32_t tl1, uint32_t mb);
'''

    # ---------------------------------------------------------------- per-quad specializations (namespace scope)
    def cls4(self, q):
        if ILP:
            return self.cls4_ilp(q)
        # GE into VCC (e32), LE into a compiler SGPR pair (e64), then the LE mask through VCC by an SALU move: a
        # VALU write of VCC read as a constant by the next VALU needs one wait state (gfx9 "mixed use of VCC"),
        # which the LE compare provides; an SALU write of VCC needs none
        L = []
        for r in range(4 * q, 4 * q + 4):
            ln = r & 63
            L += [f"v_cmp_ngt_f64 vcc, %[p], {self.reg(r)} ;@vfix 2", f"v_cmp_nlt_f64_e64 %[m], %[p], {self.reg(r)} ;@vfix 2",
                  f"v_writelane_b32 %[a0], vcc_lo, {ln}", f"v_writelane_b32 %[a1], vcc_hi, {ln}", "s_mov_b64 vcc, %[m]",
                  f"v_writelane_b32 %[a2], vcc_lo, {ln}", f"v_writelane_b32 %[a3], vcc_hi, {ln}"]
        return (f"template <> __device__ __forceinline__ void {self.name}::cls4<{q}>(double p, uint32_t (&acc)[4]) {{\n"
                f"    uint64_t m;\n"
                f"    asm volatile(\"{asm(L)}\"\n                 : [a0] \"+v\"(acc[0]), [a1] \"+v\"(acc[1]), "
                f"[a2] \"+v\"(acc[2]), [a3] \"+v\"(acc[3]), [m] \"=&s\"(m)\n                 : [p] \"s\"(p)\n"
                f"                 : \"vcc\");\n}}\n")

    def cls4_ilp(self, q):
        # the eight compares of the quad first (e64, into eight compiler-chosen SGPR pairs: independent, they
        # pipeline), then the sixteen v_writelane by the compiler (their data sources are the pairs' halves, which
        # the asm operand syntax cannot name: a C++ lane_write per half)
        rows = list(range(4 * q, 4 * q + 4))
        L = []
        for i, r in enumerate(rows):
            L += [f"v_cmp_ngt_f64_e64 %[g{i}], %[p], {self.reg(r)} ;@vfix 2",
                  f"v_cmp_nlt_f64_e64 %[l{i}], %[p], {self.reg(r)} ;@vfix 2"]
        outs = [f'[g{i}] "=&s"(g{i})' for i in range(4)] + [f'[l{i}] "=&s"(l{i})' for i in range(4)]
        wl = []
        for i, r in enumerate(rows):
            ln = r & 63
            wl += [f"    acc[0] = lane_write(acc[0], (uint32_t)g{i}, {ln}u);",
                   f"    acc[1] = lane_write(acc[1], (uint32_t)(g{i} >> 32), {ln}u);",
                   f"    acc[2] = lane_write(acc[2], (uint32_t)l{i}, {ln}u);",
                   f"    acc[3] = lane_write(acc[3], (uint32_t)(l{i} >> 32), {ln}u);"]
        return (f"template <> __device__ __forceinline__ void {self.name}::cls4<{q}>(double p, uint32_t (&acc)[4]) {{\n"
                f"    uint64_t g0, g1, g2, g3, l0, l1, l2, l3;\n"
                f"    asm volatile(\"{asm(L)}\"\n                 : {', '.join(outs)}\n                 : [p] \"s\"(p));\n"
                + "\n".join(wl) + "\n}\n")

    def exch_ilp(self, q, side, write, edge, nr=4):
        # block 1: the rows' compares; (edge forms) the rows outside [ra, ra + len] drop their masks (scalar selects);
        # block 2: every row's slot address first (readlane of the row's base, mbcnt over the mask's halves: nr
        # independent chains that pipeline), then the exec-masked LDS accesses, the reads all in flight together
        rows = list(range(nr * q, nr * q + nr))
        cmp = "v_cmp_nlt_f64" if side == 0 else "v_cmp_ngt_f64"
        L1 = [f"{cmp} %[m{i}], {self.reg(r)}, %[p] ;@vfix 1" for i, r in enumerate(rows)]
        L2 = ["s_nop 0"]  # (a VALU write of pb just before the block -> v_readlane of it: one wait state)
        L2 += [f"v_readlane_b32 %[t{i}], %[pb], {r & 63}" for i, r in enumerate(rows)]
        L2 += [f"v_mbcnt_lo_u32_b32 %[k{i}], %[ml{i}], 0" for i in range(nr)]
        L2 += [f"v_mbcnt_hi_u32_b32 %[k{i}], %[mh{i}], %[k{i}]" for i in range(nr)]
        L2 += [(f"v_lshl_add_u32 %[k{i}], %[k{i}], 3, %[t{i}]" if side == 0 else f"v_mad_i32_i24 %[k{i}], %[k{i}], -8, %[t{i}]")
               for i in range(nr)]
        L2.append("s_mov_b64 %[sv], exec")
        for i, r in enumerate(rows):
            L2 += [f"s_mov_b64 exec, %[m{i}]",
                   f"ds_write_b64 %[k{i}], {self.reg(r)} ;@vfix 1" if write else f"ds_read_b64 %[x{i}], %[k{i}]"]
        if not write:
            L2.append("s_waitcnt lgkmcnt(0)")
            for i, r in enumerate(rows):
                L2 += [f"s_mov_b64 exec, %[m{i}]", f"v_mov_b64 {self.reg(r)}, %[x{i}] ;@vfix 0"]
        L2.append("s_mov_b64 exec, %[sv]")
        mdecl = ", ".join(f"m{i}" for i in range(nr))
        decl = f"uint64_t {mdecl}, sv;\n    uint32_t " + ", ".join(f"t{i}, k{i}" for i in range(nr)) + ";\n"
        outs2 = ['[sv] "=&s"(sv)'] + [f'[t{i}] "=&s"(t{i})' for i in range(nr)] + [f'[k{i}] "=&v"(k{i})' for i in range(nr)]
        if not write:
            decl += "    uint64_t " + ", ".join(f"x{i}" for i in range(nr)) + ";\n"
            outs2 += [f'[x{i}] "=&v"(x{i})' for i in range(nr)]
        ins2 = ['[pb] "v"(pb)'] + [f'[m{i}] "s"(m{i})' for i in range(nr)] + \
               [f'[ml{i}] "s"((uint32_t)m{i})' for i in range(nr)] + [f'[mh{i}] "s"((uint32_t)(m{i} >> 32))' for i in range(nr)]
        outs1 = ", ".join(f'[m{i}] "=&s"(m{i})' for i in range(nr))
        edge_c = "".join(f"    if ({r}u - ra > len) m{i} = 0;\n" for i, r in enumerate(rows)) if edge else ""
        name = ("src" if write else "tgt") + str(nr) + ("e" if edge else "")
        args = "double p, uint32_t pb" + (", uint32_t ra, uint32_t len" if edge else "")
        return (f"template <> __device__ __forceinline__ void {self.name}::{name}<{q}, {side}>({args}) {{\n    {decl}"
                f"    asm volatile(\"{asm(L1)}\"\n                 : {outs1}\n"
                f"                 : [p] \"s\"(p));\n{edge_c}"
                f"    asm volatile(\"{asm(L2)}\"\n                 : {', '.join(outs2)}\n                 : {', '.join(ins2)}\n"
                f"                 : \"memory\", \"scc\");\n}}\n")

    def exch(self, q, side, write, edge, nr=4):
        if ILP:
            return self.exch_ilp(q, side, write, edge, nr)
        rows = list(range(nr * q, nr * q + nr))
        cmp = "v_cmp_nlt_f64" if side == 0 else "v_cmp_ngt_f64"
        L = ["s_mov_b64 %[sv], exec"]
        L += [f"{cmp} %[m{i}], {self.reg(r)}, %[p] ;@vfix 1" for i, r in enumerate(rows)]
        if edge:
            for i, r in enumerate(rows):
                L += [f"s_sub_u32 %[t], {r}, %[ra]", "s_cmp_le_u32 %[t], %[len]", f"s_cselect_b64 %[m{i}], %[m{i}], 0"]
        for i, r in enumerate(rows):
            L += [f"v_readlane_b32 %[t], %[pb], {r & 63}", f"s_mov_b64 exec, %[m{i}]",
                  "v_mbcnt_lo_u32_b32 %[k], exec_lo, 0", "v_mbcnt_hi_u32_b32 %[k], exec_hi, %[k]",
                  "v_lshl_add_u32 %[a], %[k], 3, %[t]" if side == 0 else "v_mad_i32_i24 %[a], %[k], -8, %[t]"]
            L.append(f"ds_write_b64 %[a], {self.reg(r)} ;@vfix 1" if write else f"ds_read_b64 %[t{i}], %[a]")
        if not write:
            L.append("s_waitcnt lgkmcnt(0)")
            for i, r in enumerate(rows):
                L += [f"s_mov_b64 exec, %[m{i}]", f"v_mov_b64 {self.reg(r)}, %[t{i}] ;@vfix 0"]
        L.append("s_mov_b64 exec, %[sv]")
        outs = [f'[m{i}] "=&s"(m{i})' for i in range(nr)] + ['[sv] "=&s"(sv)', '[t] "=&s"(t)', '[k] "=&v"(k)',
                                                              '[a] "=&v"(a)']
        decl = "uint64_t " + ", ".join(f"m{i}" for i in range(nr)) + ", sv;\n    uint32_t t, k, a;\n"
        if not write:
            outs += [f'[t{i}] "=&v"(t{i})' for i in range(nr)]
            decl += "    uint64_t " + ", ".join(f"t{i}" for i in range(nr)) + ";\n"
        ins = ['[p] "s"(p)', '[pb] "v"(pb)'] + (['[ra] "s"(ra)', '[len] "s"(len)'] if edge else [])
        name = ("src" if write else "tgt") + str(nr) + ("e" if edge else "")
        args = "double p, uint32_t pb" + (", uint32_t ra, uint32_t len" if edge else "")
        return (f"template <> __device__ __forceinline__ void {self.name}::{name}<{q}, {side}>({args}) {{\n    {decl}"
                f"    asm volatile(\"{asm(L)}\"\n                 : {', '.join(outs)}\n                 : {', '.join(ins)}\n"
                f"                 : \"memory\", \"scc\");\n}}\n")

    def w1quad_ilp(self, q, side):
        # the four rows side by side: the masks and prefixes come from the compiler's readlanes (C++, before the block;
        # the asm syntax cannot name one half of an SGPR pair), then the ranks (mbcnt over the mask halves, no EXEC
        # change), the compares with Ks into their own SGPR pairs, the addresses, and only then the exec-masked LDS
        # accesses (the reads all in flight together)
        rows = list(range(4 * q, 4 * q + 4))
        pro = []
        for i, j in enumerate(rows):
            pro += [f"    const uint64_t m{i} = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(mh, {j}) << 32) | "
                    f"(uint32_t)__builtin_amdgcn_readlane(ml, {j});"]
            pro += [f"    const uint32_t t{i} = __builtin_amdgcn_readlane(pre, {j}) & 0xFFFFu;" if side == 0 else
                    f"    const uint32_t t{i} = tl1 - (__builtin_amdgcn_readlane(pre, {j}) >> 16);"]
        L = [f"v_mbcnt_lo_u32_b32 %[k{i}], %[ml{i}], 0" for i in range(4)]
        L += [f"v_mbcnt_hi_u32_b32 %[k{i}], %[mh{i}], %[k{i}]" for i in range(4)]
        L += [(f"v_add_u32 %[k{i}], %[t{i}], %[k{i}]" if side == 0 else f"v_sub_u32 %[k{i}], %[t{i}], %[k{i}]")
              for i in range(4)]
        L += [f"v_cmp_gt_u32_e64 %[c{i}], %[ks], %[k{i}]" for i in range(4)]
        L += [f"v_lshl_add_u32 %[k{i}], %[k{i}], 3, %[mb]" for i in range(4)]
        L += [f"s_and_b64 %[c{i}], %[c{i}], %[m{i}]" for i in range(4)]
        return pro, L

    def w1quad(self, q, side, write):
        rows = list(range(4 * q, 4 * q + 4))
        if ILP:
            pro, L = self.w1quad_ilp(q, side)
            L.append("s_mov_b64 %[sv], exec")
            for i, j in enumerate(rows):
                L += [f"s_mov_b64 exec, %[c{i}]",
                      f"ds_write_b64 %[k{i}], {self.reg(j)} ;@vfix 1" if write else f"ds_read_b64 %[x{i}], %[k{i}]"]
            if not write:
                L.append("s_waitcnt lgkmcnt(0)")
                for i, j in enumerate(rows):
                    L += [f"s_mov_b64 exec, %[c{i}]", f"v_mov_b64 {self.reg(j)}, %[x{i}] ;@vfix 0"]
            L.append("s_mov_b64 exec, %[sv]")
            outs = ['[sv] "=&s"(sv)'] + [f'[c{i}] "=&s"(c{i})' for i in range(4)] + [f'[k{i}] "=&v"(k{i})' for i in range(4)]
            decl = "uint64_t sv, c0, c1, c2, c3;\n    uint32_t k0, k1, k2, k3;\n"
            if not write:
                outs += [f'[x{i}] "=&v"(x{i})' for i in range(4)]
                decl += "    uint64_t x0, x1, x2, x3;\n"
            ins = [f'[m{i}] "s"(m{i})' for i in range(4)] + [f'[ml{i}] "s"((uint32_t)m{i})' for i in range(4)] + \
                  [f'[mh{i}] "s"((uint32_t)(m{i} >> 32))' for i in range(4)] + [f'[t{i}] "s"(t{i})' for i in range(4)] + \
                  ['[ks] "s"(ks)', '[mb] "s"(mb)']
            name = "w1src" if write else "w1tgt"
            return (f"template <> __device__ __forceinline__ void {self.name}::{name}<{q}, {side}>(uint32_t ml, uint32_t mh, "
                    f"uint32_t pre, uint32_t ks, uint32_t tl1, uint32_t mb) {{\n" + "\n".join(pro) + f"\n    {decl}"
                    f"    asm volatile(\"{asm(L)}\"\n                 : {', '.join(outs)}\n                 : {', '.join(ins)}\n"
                    f"                 : \"memory\", \"scc\");\n}}\n")
        L = ["s_nop 0"]  # (a VALU write of ml / mh / pre just before the block -> v_readlane of it: one wait state)
        for i, j in enumerate(rows):
            L += [f"v_readlane_b32 vcc_lo, %[ml], {j}", f"v_readlane_b32 vcc_hi, %[mh], {j}",
                  f"v_readlane_b32 %[t], %[pre], {j}"]
            L += ["s_and_b32 %[t], %[t], 0xffff"] if side == 0 else ["s_lshr_b32 %[t], %[t], 16", "s_sub_u32 %[t], %[tl1], %[t]"]
            L += ["s_and_saveexec_b64 %[sv], vcc", "v_mbcnt_lo_u32_b32 %[k], exec_lo, 0",
                  "v_mbcnt_hi_u32_b32 %[k], exec_hi, %[k]",
                  "v_add_u32 %[k], %[t], %[k]" if side == 0 else "v_sub_u32 %[k], %[t], %[k]",
                  "v_cmp_gt_u32 vcc, %[ks], %[k]", "s_and_b64 exec, exec, vcc", "v_lshl_add_u32 %[a], %[k], 3, %[mb]"]
            if write:
                L += [f"ds_write_b64 %[a], {self.reg(j)} ;@vfix 1", "s_mov_b64 exec, %[sv]"]
            else:
                L += [f"ds_read_b64 %[x{i}], %[a]", f"s_mov_b64 %[m{i}], exec", "s_mov_b64 exec, %[sv]"]
        if not write:
            L.append("s_waitcnt lgkmcnt(0)")
            for i, j in enumerate(rows):
                L += [f"s_and_saveexec_b64 %[sv], %[m{i}]", f"v_mov_b64 {self.reg(j)}, %[x{i}] ;@vfix 0",
                      "s_mov_b64 exec, %[sv]"]
        outs = ['[sv] "=&s"(sv)', '[t] "=&s"(t)', '[k] "=&v"(k)', '[a] "=&v"(a)']
        decl = "uint64_t sv;\n    uint32_t t, k, a;\n"
        if not write:
            outs += [f'[m{i}] "=&s"(m{i})' for i in range(4)] + [f'[x{i}] "=&v"(x{i})' for i in range(4)]
            decl += "    uint64_t m0, m1, m2, m3, x0, x1, x2, x3;\n"
        ins = ['[ml] "v"(ml)', '[mh] "v"(mh)', '[pre] "v"(pre)', '[ks] "s"(ks)', '[tl1] "s"(tl1)', '[mb] "s"(mb)']
        name = "w1src" if write else "w1tgt"
        return (f"template <> __device__ __forceinline__ void {self.name}::{name}<{q}, {side}>(uint32_t ml, uint32_t mh, "
                f"uint32_t pre, uint32_t ks, uint32_t tl1, uint32_t mb) {{\n    {decl}"
                f"    asm volatile(\"{asm(L)}\"\n                 : {', '.join(outs)}\n                 : {', '.join(ins)}\n"
                f"                 : \"memory\", \"scc\", \"vcc\");\n}}\n")

    def specializations(self):
        out = []
        for q in range(self.rows // 4):
            out.append(self.cls4(q))
            for s in (0, 1):
                for e in (False, True):
                    out.append(self.exch(q, s, True, e))
                    out.append(self.exch(q, s, False, e))
        if self.name == "RowsA":  # (targets of a wholly covered quad pair: eight reads in flight; LayA has the registers)
            for o in range(self.rows // 8):
                for s in (0, 1):
                    out.append(self.exch(o, s, False, False, nr=8))
        for q in range(W1QUADS):
            for s in (0, 1):
                out.append(self.w1quad(q, s, True))
                out.append(self.w1quad(q, s, False))
        return out


def main(out=OUT):
    parts = ["// refv_rows.h -- GENERATED by tools/gen_refv_rows.py; do not edit.",
             "// K2V's asm on its fixed data registers, one struct per register layout (see the generator's docstring).",
             "// Included inside align_refv.hip's namespace.", "#pragma once", ""]
    gens = [Gen(n, b) for n, b in LAYOUTS]
    for g in gens:
        parts.append(f"struct {g.name} {{\n{g.members()}}};\n")
    for g in gens:
        parts += g.specializations()
    with open(out, "w") as f:
        f.write("\n".join(parts))
    print("wrote", out)


if __name__ == "__main__":
    # (an explicit path writes there instead: tests/test_asm_checks.py regenerates the header and diffs it)
    import sys
    main(sys.argv[1] if len(sys.argv) > 1 else OUT)
