"""Generates pitt_object_table_segmentation_amd/csrc/score_list_asm.inc: the hand-scheduled gfx950
loop that scores one group's compacted survivor list in k_score.

    python tools/gen_score_asm.py

One inline-asm block per PCL reduction order (A3).  Entry k of the list (a float4 plane row at LDS
byte address base + 16 k) is scored against the group's 64 points (one per lane) in PCL's exact
float order -- 3 v_mul + 3 v_add, no FMA -- then |d| < t by v_cmp, s_bcnt1 of the mask, and the
count is written to lane L + k of vc with an immediate lane select.  Two entries per step with the
next two rows already in flight; an odd-length list runs a single-entry head first so no step
scores a padding row.  Coefficient rows live in the fixed registers v[56:71] (clobbered).
"""
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "pitt_object_table_segmentation_amd", "csrc", "score_list_asm.inc")
REGS = [56, 60, 64, 68]  # four float4 row registers: two in use, two in flight
NMAX = 16  # list length of the block being generated


def comp(r, k):
    return f"v{r + k}"


def dot(order, d, t, r):
    """PCL's 4-lane dot (c.x x, c.y y, c.z z, c.w) in reduction order `order` into d (t scratch)."""
    a0, a1, a2, a3 = (comp(r, k) for k in range(4))
    if order == 0:    # SSE2: (a0 + a2) + (a1 + a3)
        return [f"v_mul_f32 {d}, {a0}, %[x]", f"v_mul_f32 {t}, {a2}, %[z]", f"v_add_f32 {d}, {d}, {t}",
                f"v_mul_f32 {t}, {a1}, %[y]", f"v_add_f32 {t}, {t}, {a3}", f"v_add_f32 {d}, {d}, {t}"]
    if order == 1:    # SSE3 hadd: (a0 + a1) + (a2 + a3)
        return [f"v_mul_f32 {d}, {a0}, %[x]", f"v_mul_f32 {t}, {a1}, %[y]", f"v_add_f32 {d}, {d}, {t}",
                f"v_mul_f32 {t}, {a2}, %[z]", f"v_add_f32 {t}, {t}, {a3}", f"v_add_f32 {d}, {d}, {t}"]
    # sequential: ((a0 + a1) + a2) + a3
    return [f"v_mul_f32 {d}, {a0}, %[x]", f"v_mul_f32 {t}, {a1}, %[y]", f"v_add_f32 {d}, {d}, {t}",
            f"v_mul_f32 {t}, {a2}, %[z]", f"v_add_f32 {d}, {d}, {t}", f"v_add_f32 {d}, {d}, {a3}"]


def rd(r, off):
    return f"ds_read_b128 v[{r}:{r + 3}], %[base] offset:{off}"


def wl(src, k):
    """entry k's count into lane L + k of vc (k < 16) or lane L + k - 16 of vc2 (32-entry lists)"""
    return f"v_writelane_b32 %[vc], {src}, %[L]+{k}" if k < 16 else f"v_writelane_b32 %[vc2], {src}, %[L]+{k - 16}"


def single(order, r, k):
    out = dot(order, "%[d0]", "%[t0]", r)
    out += ["v_cmp_lt_f32 %[m0], |%[d0]|, %[tv]", "s_bcnt1_i32_b64 %[n0], %[m0]", wl("%[n0]", k)]
    return out


def pair(order, ra, rb, k):
    a, b = dot(order, "%[d0]", "%[t0]", ra), dot(order, "%[d1]", "%[t1]", rb)
    out = [x for ab in zip(a, b) for x in ab]  # two independent chains, interleaved
    out += ["v_cmp_lt_f32 %[m0], |%[d0]|, %[tv]", "v_cmp_lt_f32 %[m1], |%[d1]|, %[tv]",
            "s_bcnt1_i32_b64 %[n0], %[m0]", "s_bcnt1_i32_b64 %[n1], %[m1]", wl("%[n0]", k), wl("%[n1]", k + 1)]
    return out


def block(order, nmax=16):
    global NMAX
    NMAX = nmax
    out = []
    # odd c: entry 0 alone, then pairs from entry 1
    out += ["s_bitcmp1_b32 %[c], 0", "s_cbranch_scc0 .Leven%="]
    out += [rd(REGS[0], 0), rd(REGS[1], 16), rd(REGS[2], 32), "s_waitcnt lgkmcnt(2)"]
    out += single(order, REGS[0], 0)
    out += ["s_cmp_le_u32 %[c], 1", "s_cbranch_scc1 .Lwait%="]
    # rows of entries 1, 2 are in REGS[1], REGS[2]: rotate so the pair path starts there
    odd = path_from(order, 1, [REGS[1], REGS[2], REGS[3], REGS[0]], prefetched=True)
    out += odd
    out += ["s_branch .Lwait%=", ".Leven%=:"]
    out += [rd(REGS[0], 0), rd(REGS[1], 16)]
    out += path_from(order, 0, REGS[:], prefetched=False)
    out += [".Lwait%=:", "s_waitcnt lgkmcnt(0)"]
    return out


def path_from(order, first, regs, prefetched):
    """Pairs from entry `first`; rows of first, first+1 are read (or in flight) in regs[0], regs[1].
    prefetched: one more read (first+1) than the pair is outstanding after the head entry."""
    out = []
    k = first
    regs = regs[:]
    n = NMAX
    while k < n:
        ra, rb, rc, rd_ = regs
        if k + 2 < n:
            out += [rd(rc, 16 * (k + 2))]
            if k + 3 < n:
                out += [rd(rd_, 16 * (k + 3))]
                out += ["s_waitcnt lgkmcnt(2)"]
            else:
                out += ["s_waitcnt lgkmcnt(1)"]
        else:
            out += ["s_waitcnt lgkmcnt(0)"]
        if k + 1 < n:
            out += pair(order, ra, rb, k)
        else:
            out += single(order, ra, k)
        if k + 2 < n:
            out += [f"s_cmp_le_u32 %[c], {k + 2}", "s_cbranch_scc1 .Lwait%="]
        regs = [rc, rd_, ra, rb]
        k += 2
    return out


# ---- software-pipelined walk: the count chain of one pair (v_cmp -> s_bcnt1 -> v_writelane, a
# VALU -> SALU -> VALU round trip) runs interleaved with the next pair's dot products, so a wave does
# not stall on it.  Registers: the pairs' results alternate between (d0, d1) and (e0, e1); t0, t1 are
# the dots' scratch.  Same operations per entry as pair() / single(), so the counts are the same bits.
def dots_pair(order, ra, rb, ra_out, rb_out):
    a, b = dot(order, ra_out, "%[t0]", ra), dot(order, rb_out, "%[t1]", rb)
    return [x for ab in zip(a, b) for x in ab]


def chain_parts(x0, x1, k):
    cmps = [f"v_cmp_lt_f32 %[m0], |{x0}|, %[tv]", f"v_cmp_lt_f32 %[m1], |{x1}|, %[tv]"]
    rest = ["s_bcnt1_i32_b64 %[n0], %[m0]", "s_bcnt1_i32_b64 %[n1], %[m1]", wl("%[n0]", k), wl("%[n1]", k + 1)]
    return cmps, rest


def interleave(rest, dots):
    """bcnt0 after 4 dot ops, bcnt1 after 6, writelane0 after 8, writelane1 after 10"""
    out = []
    marks = {4: rest[0], 6: rest[1], 8: rest[2], 10: rest[3]}
    for i, ins in enumerate(dots):
        if i in marks:
            out.append(marks[i])
        out.append(ins)
    return out


def path_from_pipe(order, first, regs, tag):
    """As path_from, pipelined: pair (k, k+1)'s dots, then for every later pair its reads, the previous
    pair's compares, the LDS wait, and its dots interleaved with the previous pair's counts.  An exit
    after pair j jumps to .Lf<tag><j>, which finishes pair j's counts."""
    out, tails = [], []
    n = NMAX
    k = first
    ra, rb, rc, rd_ = regs
    names = [("%[d0]", "%[d1]"), ("%[e0]", "%[e1]")]
    cur = 0

    def reads(k, rc, rd_):
        r = []
        if k + 2 < n:
            r.append(rd(rc, 16 * (k + 2)))
            if k + 3 < n:
                r.append(rd(rd_, 16 * (k + 3)))
                return r, "s_waitcnt lgkmcnt(2)"
            return r, "s_waitcnt lgkmcnt(1)"
        return r, "s_waitcnt lgkmcnt(0)"

    if k + 1 >= n:  # a lone last entry: not reached by any list of a valid length
        r, w = reads(k, rc, rd_)
        return out + r + [w] + single(order, ra, k), tails
    r, w = reads(k, rc, rd_)
    out += r + [w] + dots_pair(order, ra, rb, *names[cur])
    while True:
        x0, x1 = names[cur]
        cmps, rest = chain_parts(x0, x1, k)
        if k + 2 >= n:
            out += cmps + rest
            break
        lab = f".Lf{tag}{k}_%="
        out += [f"s_cmp_le_u32 %[c], {k + 2}", f"s_cbranch_scc1 {lab}"]
        tails += [f"{lab}:"] + cmps + rest + ["s_branch .Lwait%="]
        k += 2
        ra, rb, rc, rd_ = rc, rd_, ra, rb
        r, w = reads(k, rc, rd_)
        if k + 1 >= n:  # the last entry of a maximal odd-path list alone (never reached)
            out += r + cmps + [w] + rest + single(order, ra, k)
            break
        nxt = 1 - cur
        out += r + cmps + [w] + interleave(rest, dots_pair(order, ra, rb, *names[nxt]))
        cur = nxt
    return out, tails


def block_pipe(order, nmax=16):
    global NMAX
    NMAX = nmax
    out = []
    out += ["s_bitcmp1_b32 %[c], 0", "s_cbranch_scc0 .Leven%="]
    out += [rd(REGS[0], 0), rd(REGS[1], 16), rd(REGS[2], 32), "s_waitcnt lgkmcnt(2)"]
    out += single(order, REGS[0], 0)
    out += ["s_cmp_le_u32 %[c], 1", "s_cbranch_scc1 .Lwait%="]
    odd, t1 = path_from_pipe(order, 1, [REGS[1], REGS[2], REGS[3], REGS[0]], "o")
    out += odd
    out += ["s_branch .Lwait%=", ".Leven%=:"]
    out += [rd(REGS[0], 0), rd(REGS[1], 16)]
    even, t2 = path_from_pipe(order, 0, REGS[:], "e")
    out += even
    out += ["s_branch .Lwait%="] + t1 + t2
    out += [".Lwait%=:", "s_waitcnt lgkmcnt(0)"]
    return out


def main():
    lines = ["// GENERATED by tools/gen_score_asm.py -- do not edit by hand.",
             "// k_score's survivor-list loop for one group, per PCL reduction order (A3); see the generator's",
             "// docstring for the schedule.  Operands: base (VGPR, LDS byte address of entry 0), c (SGPR,",
             "// 1..16 entries), x, y, z, tv (VGPRs), vc (VGPR, in/out), L (immediate lane base 16 g);",
             "// d0, t0, d1, t1 (VGPR scratch), m0, m1 (SGPR pairs), n0, n1 (SGPRs).  Clobbers v56-v71.",
             "#pragma once", ""]
    for nmax, name, gen in ((16, "PITT_SCORE_LIST_ASM", block), (32, "PITT_SCORE_LIST32_ASM", block),
                            (16, "PITT_SCORE_LIST_ASM_P", block_pipe), (32, "PITT_SCORE_LIST32_ASM_P", block_pipe)):
        if nmax == 32 and gen is block:
            lines.append("// 32-entry lists (two rounds of hypotheses in one pass): entries 16.. write lane L + k - 16 of vc2.")
        if name.endswith("_P") and nmax == 16:
            lines.append("// _P: the same walks software-pipelined (a pair's count chain under the next pair's dots;")
            lines.append("// e0, e1 VGPR scratch as well).")
        for order in range(3):
            body = gen(order, nmax)
            lines.append(f"#define {name}_{order} \\")
            for i, ins in enumerate(body):
                end = " \\" if i + 1 < len(body) else ""
                lines.append(f'    "{ins}\\n"{end}')
            lines.append("")
    open(OUT, "w").write("\n".join(lines) + "\n")
    print(f"wrote {OUT}: {len(block(0))} / {len(block(0, 32))} instructions per order (16 / 32 entries)")


if __name__ == "__main__":
    main()
