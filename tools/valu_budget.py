"""Per-phase VALU budget of one kernel from its gfx950 ISA (analysis only, CPU).

The kernel's body is cut into phases at its `s_barrier` instructions (one phase per barrier-delimited region, in
program order).  Each VALU instruction is weighted by its issue class on gfx950 (profiles/r05_valu_issue_rates.txt,
tools/micro/valu_rate.hip): 2 cycles for the VOP2/VOP1 32-bit integer / logic / f32 forms, the VOP2 16-bit max / min
/ add and v_mov; 4 cycles for every packed op, every 3-input op, 32-bit max / min, v_lshlrev, 24/32-bit multiplies,
v_mbcnt, v_cmp, VOP3 cndmask, conversions, readlane / readfirstlane, SDWA and DPP forms.  Loop bodies (basic blocks
the compiler marks "in Loop") are listed with their own counts, so a dynamic budget is static count x trip count.

    python tools/valu_budget.py /tmp/isa_orb_extract.s og_fast_quad_kernel
    (the .s comes from: bash tools/isa.sh orb_extract.hip)
"""
import re
import sys

TWO = re.compile(r"^v_(add|sub|subrev)_(u32|i32|f32|co_u32)(_e32)?$|^v_(and|or|xor)_b32(_e32)?$|^v_lshrrev_b32(_e32)?$|"
                 r"^v_ashrrev_i32(_e32)?$|^v_(mul|fma|fmac|mac)_f32(_e32)?$|^v_(max|min|add|sub)_(u16|i16|f16)(_e32)?$|"
                 r"^v_mov_b32(_e32)?$|^v_not_b32(_e32)?$|^v_cndmask_b32_e32$")


def classify(op: str, line: str) -> int:
    """Issue cycles of one wave64 VALU instruction (2 or 4)."""
    if " sdwa" in line or "dpp" in line or "row_" in line or "quad_perm" in line:
        return 4
    return 2 if TWO.match(op) else 4


def kernel_body(asm: str, name: str) -> str:
    m = re.search(r"^(_Z\w*" + re.escape(name) + r"\w*):", asm, re.M)
    if not m:
        raise SystemExit(f"kernel {name} not in the assembly")
    end = asm.index(".Lfunc_end", m.end())
    return asm[m.end():end]


def phases(body: str):
    out, cur = [], {"lines": [], "blocks": []}
    block = ("entry", False)
    for raw in body.split("\n"):
        t = raw.strip()
        if not t or t.startswith((";", ".")) and not re.match(r"^\.LBB\d+_\d+:", t):
            if t.startswith("; %bb."):
                block = (t.split()[1].rstrip(":"), "Loop" in t)
            continue
        lm = re.match(r"^(\.LBB\d+_\d+):(.*)$", t)
        if lm:
            block = (lm.group(1), "Loop" in lm.group(2))
            continue
        op = t.split()[0]
        cur["lines"].append((block, op, t))
        if op == "s_barrier":
            out.append(cur)
            cur = {"lines": [], "blocks": []}
    out.append(cur)
    return out


def summarise(ph):
    rows = []
    for k, p in enumerate(ph):
        blocks = {}
        order = []
        for (bname, loop), op, t in p["lines"]:
            if not op.startswith("v_"):
                continue
            key = (bname, loop)
            if key not in blocks:
                blocks[key] = [0, 0]
                order.append(key)
            c = classify(op, t)
            blocks[key][0] += 1
            blocks[key][1] += c
        n = sum(v[0] for v in blocks.values())
        cyc = sum(v[1] for v in blocks.values())
        rows.append((k, n, cyc, [(b, l, blocks[(b, l)][0], blocks[(b, l)][1]) for b, l in order]))
    return rows


def main():
    path, name = sys.argv[1], sys.argv[2]
    body = kernel_body(open(path).read(), name)
    ph = phases(body)
    print(f"# {name}: static VALU per barrier-delimited phase (count / issue cycles, 2- and 4-cycle classes)")
    tot_n = tot_c = 0
    for k, n, cyc, blocks in summarise(ph):
        tot_n += n
        tot_c += cyc
        print(f"phase {k}: {n} VALU, {cyc} cycles")
        for b, loop, bn, bc in blocks:
            print(f"    {b:10s} {'loop ' if loop else '     '} {bn:4d} VALU {bc:5d} cycles")
    print(f"total: {tot_n} VALU, {tot_c} cycles")


if __name__ == "__main__":
    main()
