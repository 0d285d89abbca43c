"""SGPR write-after-read distances for vector-memory instructions (diagnostic):
for every buffer/global load or store that reads an SGPR (soffset or the
resource / address base), the number of instructions until the next
instruction that WRITES that SGPR (layout order inside basic blocks).
usage: python tools/r3/sgpr_war.py <listing.s> <kernel symbol>"""
import re
import sys
from collections import Counter


def sregs(tok):
    m = re.fullmatch(r"s\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.fullmatch(r"s(\d+)", tok)
    return {int(m.group(1))} if m else set()


def main(path, sym):
    lines = open(path).read().splitlines()
    st = next(i for i, l in enumerate(lines) if l.startswith(sym + ":"))
    pend = {}          # sgpr -> (instr index, text)
    hist = Counter()
    ex = []
    n = 0
    for l in lines[st + 1:]:
        if l.startswith(".Lfunc_end"):
            break
        s = l.split(";")[0].strip()
        if not s or s.startswith("."):
            if s.startswith(".LBB"):
                pend.clear()
            continue
        op, _, rest = s.partition(" ")
        ops = [w for t in rest.split(",") for w in t.split()] if rest else []
        if op.startswith(("buffer_", "global_")):
            for t in ops:
                for r in sregs(t):
                    pend[r] = (n, s)
        elif op.startswith(("s_", "v_readlane", "v_readfirstlane")) and ops and \
                not op.startswith(("s_waitcnt", "s_nop", "s_barrier", "s_branch", "s_cbranch",
                                   "s_cmp", "s_endpgm", "s_setprio", "s_bitcmp")):
            for r in sregs(ops[0]):
                if r in pend:
                    d = n - pend[r][0]
                    hist[d] += 1
                    if d <= 3:
                        ex.append((d, s, pend[r][1]))
                    del pend[r]
        n += 1
    print("VMEM SGPR read -> SALU overwrite distance (instructions):", sorted(hist.items())[:12])
    for d, a, b in ex[:8]:
        print(f"  {d}: {a}   <- {b}")
    print(f"  {len(ex)} overwrites within 3 instructions")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
