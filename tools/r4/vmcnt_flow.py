"""Path-insensitive dataflow check of vmcnt coverage (diagnostic; round 4).

Unlike tools/r3/vmcnt_sim.py (one simulated path, masked blocks always
executed), this explores EVERY control-flow edge: an `s_cbranch_execz` block
is skipped by a wave whose exec is empty (e.g. the bias-staging block only
wave 0 runs), so its `s_waitcnt vmcnt(0)` does not drain the other waves'
queues.  State per program point: for every VGPR/AGPR with a load still
possibly in flight, the fewest vector-memory operations issued after that
load on any path ("younger" count).  `s_waitcnt vmcnt(N)` retires entries
with younger >= N; every VMEM op increments all counts.  Loads, stores and
LDS-DMA count alike, in issue order (MI355X_MICROARCH.md).  Reports every
read (or non-VMEM write) of a register whose load may still be in flight.

usage: python tools/r4/vmcnt_flow.py <listing.s> <kernel symbol>
"""
import re
import sys

CAP = 64


def regs(tok):
    m = re.fullmatch(r"([va])\[(\d+):(\d+)\]", tok)
    if m:
        return {(m.group(1), i) for i in range(int(m.group(2)), int(m.group(3)) + 1)}
    m = re.fullmatch(r"-?\|?([va])(\d+)\|?", tok)
    if m:
        return {(m.group(1), int(m.group(2)))}
    return set()


def parse(path, sym):
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if l.startswith(sym + ":"))
    body, labels = [], {}
    for l in lines[start + 1:]:
        s = l.split(";")[0].strip()
        if s.startswith(".Lfunc_end"):
            break
        if not s or (s.startswith(".") and not s.startswith(".LBB")):
            continue
        if s.endswith(":"):
            labels[s[:-1]] = len(body)
            continue
        op, _, rest = s.partition(" ")
        ops = [t.strip() for t in rest.split(",")] if rest else []
        body.append((op, ops, l.strip()))
    return body, labels


def succs(body, labels, pc):
    op, ops, _ = body[pc]
    if op == "s_endpgm":
        return []
    if op == "s_branch":
        return [labels[ops[0]]]
    if op.startswith("s_cbranch"):
        return [labels[ops[0]], pc + 1]
    return [pc + 1]


def step(body, pc, st, report):
    op, ops, text = body[pc]
    if op == "s_waitcnt":
        m = re.search(r"vmcnt\((\d+)\)", text)
        if m:
            n = int(m.group(1))
            st = {r: y for r, y in st.items() if y < n}
        return st
    is_load = op.startswith(("buffer_load", "global_load", "flat_load", "scratch_load"))
    is_lds_dma = is_load and " lds" in text
    is_vm = is_load or op.startswith(("buffer_store", "global_store", "flat_store",
                                      "scratch_store", "global_atomic", "buffer_atomic"))
    srcs, dsts = set(), set()
    if is_load:
        for t in ops[1:]:
            srcs |= regs(t)
        if not is_lds_dma and ops:
            dsts = regs(ops[0])
    elif op.startswith(("ds_write", "global_store", "buffer_store", "flat_store", "v_cmp",
                        "v_readlane", "v_readfirstlane", "s_")):
        for t in ops:
            srcs |= regs(t)
    elif op.startswith(("v_", "ds_")):
        for t in ops[1:]:
            srcs |= regs(t)
        if ops:
            dsts = regs(ops[0])
    bad = srcs & set(st)
    if bad:
        report.append((pc, "RAW", text, sorted(bad)[:4]))
    if not is_load:
        wb = dsts & set(st)
        if wb:
            report.append((pc, "WAW", text, sorted(wb)[:4]))
    if is_vm:
        st = {r: min(y + 1, CAP) for r, y in st.items()}
    if is_load and dsts:
        st = dict(st)
        for r in dsts:
            st[r] = 0
    return st


def merge(a, b):
    out = dict(a)
    for r, y in b.items():
        out[r] = min(out.get(r, CAP), y)
    return out


def main():
    body, labels = parse(sys.argv[1], sys.argv[2])
    state_in = {0: {}}
    work = [0]
    while work:
        pc = work.pop()
        st = step(body, pc, state_in[pc], [])
        for s in succs(body, labels, pc):
            if s >= len(body):
                continue
            new = merge(state_in[s], st) if s in state_in else st
            if s not in state_in or new != state_in[s]:
                state_in[s] = new
                work.append(s)
    report = []
    for pc in sorted(state_in):
        step(body, pc, state_in[pc], report)
    print(f"{len(body)} instructions, {len(report)} possible reads/writes of in-flight loads")
    for pc, kind, text, r in report[:60]:
        print(f"  @{pc} {kind}: {text[:90]}   regs {r}")


if __name__ == "__main__":
    main()
