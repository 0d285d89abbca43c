"""Scan an ISA listing for the VMEM -> SALU SGPR write-after-read pattern that
root-caused the K-split co-residency fault (round 4): a
vector-memory instruction reads an SGPR (soffset, the buffer resource, the
saddr base, or M0 for LDS-DMA) and an SALU / SMEM instruction rewrites that
SGPR fewer than WS wait states later.  Counts per kernel.

usage: python tools/r4/sgpr_war_scan.py <listing.s> [WS=8]
"""
import re
import sys
from collections import defaultdict


def sgprs(tok):
    m = re.fullmatch(r"s\[(\d+):(\d+)\]", tok)
    if m:
        return {f"s{i}" for i in range(int(m.group(1)), int(m.group(2)) + 1)}
    if re.fullmatch(r"s\d+|m0|vcc|exec", tok):
        return {tok}
    return set()


def wait_states(op, t):
    if op == "s_nop":
        return int(t.split()[1]) + 1
    return 1


def scan(path, ws=8):
    out = defaultdict(int)
    fn = None
    recent = []     # [(sgprs read, states since)]
    for l in open(path):
        s = l.split(";")[0].strip()
        if re.match(r"^_Z\w+:$", s):
            fn, recent = s[:-1], []
            continue
        if not s or s.startswith(".") and not s.startswith(".LBB"):
            continue
        if s.endswith(":"):
            recent = []          # conservatively restart at labels
            continue
        op, _, rest = s.partition(" ")
        toks = [x for x in re.split(r"[,\s]+", rest) if x]
        if op.startswith(("s_", "v_readfirstlane", "v_readlane")) and toks and \
                op not in ("s_nop", "s_waitcnt", "s_barrier", "s_endpgm", "s_setprio") and \
                not op.startswith(("s_cbranch", "s_branch", "s_sleep", "s_waitcnt")):
            dst = sgprs(toks[0]) if not op.startswith(("s_cmp", "s_bitcmp")) else set()
            if op.startswith("s_") and op.endswith(("_saveexec_b64", "_saveexec_b32")):
                dst |= {"exec"}
            for rd, st in recent:
                if dst & rd and st < ws:
                    out[fn] += 1
                    break
        n = wait_states(op, s)
        recent = [(rd, st + n) for rd, st in recent if st + n < ws]
        if op.startswith(("buffer_", "global_", "scratch_")):
            rd = set()
            for t in toks:
                rd |= sgprs(t)
            if " lds" in s:
                rd |= {"m0"}
            recent.append((rd, 0))
    return out


if __name__ == "__main__":
    ws = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    for fn, n in sorted(scan(sys.argv[1], ws).items(), key=lambda x: -x[1]):
        print(f"{n:5d}  {fn}")
