"""Static check of vmcnt coverage in a gfx9 ISA listing (diagnostic).

Walks one kernel's instruction stream along its control flow (exec-masked
blocks taken, loop back-edges followed a bounded number of times), keeps the
queue of outstanding vector-memory operations (loads / stores / LDS-DMA count
together, in issue order; `s_waitcnt vmcnt(N)` retires all but the N youngest)
and reports every instruction that reads a VGPR whose load is still pending.
usage: python tools/r3/vmcnt_sim.py <listing.s> <kernel symbol> [max_loop_iters]"""
import re
import sys

def regs(tok):
    """VGPR / AGPR indices named by one operand token."""
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
        if not s or s.startswith(".") and not s.startswith(".LBB"):
            if s.startswith(".Lfunc_end"):
                break
            continue
        if s.endswith(":"):
            labels[s[:-1]] = len(body)
            continue
        op, _, rest = s.partition(" ")
        ops = [t.strip() for t in rest.split(",")] if rest else []
        body.append((op, ops, l.strip()))
        if op == "s_endpgm":
            pass
    return body, labels


def simulate(body, labels, max_iters=2):
    pending = []          # (pc, kind, dst regs)
    hazards = []
    visits = {}
    pc = 0
    steps = 0
    while pc < len(body) and steps < 2_000_000:
        steps += 1
        op, ops, text = body[pc]
        if op == "s_endpgm":
            break
        if op == "s_waitcnt":
            m = re.search(r"vmcnt\((\d+)\)", text)
            if m:
                n = int(m.group(1))
                while len(pending) > n:
                    pending.pop(0)
            pc += 1
            continue
        is_vmem_load = op.startswith(("buffer_load", "global_load", "flat_load", "scratch_load"))
        is_vmem_store = op.startswith(("buffer_store", "global_store", "flat_store", "scratch_store",
                                       "global_atomic", "buffer_atomic"))
        # sources
        srcs = set()
        if is_vmem_load:
            for t in ops[1:]:
                srcs |= regs(t)
        elif op.startswith(("v_", "ds_", "global_store", "buffer_store", "flat_store")):
            first = 0 if (op.startswith(("ds_write", "global_store", "buffer_store", "flat_store"))
                          or op.startswith("v_cmp") or op.startswith("v_readlane")
                          or op.startswith("v_readfirstlane")) else 1
            for t in ops[first:]:
                srcs |= regs(t)
        live = {r: p for p in pending if p[1] == "load" for r in p[2]}
        bad = srcs & set(live)
        if bad:
            hazards.append((pc, "RAW " + text, sorted(bad)[:4], live[sorted(bad)[0]][0]))
        # write-after-write: a non-VMEM write of a register whose load is still pending
        if not is_vmem_load and ops and (op.startswith("v_") or op.startswith("ds_read")) \
                and not op.startswith(("v_cmp", "v_readlane", "v_readfirstlane")):
            wb = regs(ops[0]) & set(live)
            if wb:
                hazards.append((pc, "WAW " + text, sorted(wb)[:4], live[sorted(wb)[0]][0]))
        if is_vmem_load:
            pending.append((pc, "load", regs(ops[0]) if ops else set()))
        elif is_vmem_store:
            pending.append((pc, "store", set()))
        elif op.startswith(("v_", "ds_read")) and ops:
            # a VALU / LDS write of a register an outstanding load also targets: drop tracking (WAW)
            pass
        # control flow
        if op == "s_branch":
            tgt = ops[0]
            visits[tgt] = visits.get(tgt, 0) + 1
            pc = labels[tgt]
            continue
        if op.startswith("s_cbranch"):
            tgt = ops[0]
            if pc + 1 < len(body) and body[pc + 1][0] == "s_endpgm" and labels[tgt] > pc:
                pc = labels[tgt]                 # the early-exit guard: take the working path
                continue
            if op in ("s_cbranch_execz", "s_cbranch_execnz") or "vcc" in op:
                pc += 1                      # masked block: fall through (executed in order)
                continue
            # scc branches (loop control): take a back-edge up to max_iters, else fall through
            key = (pc, tgt)
            if labels[tgt] < pc:
                visits[key] = visits.get(key, 0) + 1
                pc = labels[tgt] if visits[key] < max_iters else pc + 1
            else:
                visits[key] = visits.get(key, 0) + 1
                pc = labels[tgt] if visits[key] >= max_iters else pc + 1
            continue
        pc += 1
    return hazards, steps


if __name__ == "__main__":
    body, labels = parse(sys.argv[1], sys.argv[2])
    hz, steps = simulate(body, labels, int(sys.argv[3]) if len(sys.argv) > 3 else 2)
    print(f"{len(body)} instructions, {steps} simulated, {len(hz)} reads of pending loads")
    for pc, text, r, src in hz[:40]:
        print(f"  @{pc}: {text}   regs {r} loaded @{src}: {body[src][2]}")
