"""ISA-level bisection patches for the K-split forward-only (MODE 1) kernel
(diagnostic only).  Reads the part-6 kind-1 assembly of a
NERFHIP_EXP_KS_MODES build, applies one patch inside
k_step_rows_ks<256,128,1> only, writes the patched file.

  python tools/r4/ks_patch.py <in.s> <out.s> <patch>

Regions (labels of that function in the emitted assembly): the FINAL phase
runs from the last `s_cbranch_scc0` join before the final-phase MFMAs (the
first instruction after the hidden-layer loop exit) to s_endpgm.
"""
import re
import sys

src = open(sys.argv[1]).read().split("\n")
out_path, patch = sys.argv[2], sys.argv[3]
import os
name = os.environ.get("KS_SYM", "_ZN12_GLOBAL__N_114k_step_rows_ksILi256ELi128ELi1EEEvN14nerfhip_detail5KArgsE")
s = next(i for i, l in enumerate(src) if l.startswith(name + ":"))
e = next(i for i in range(s, len(src)) if src[i].strip().startswith(".Lfunc_end")) - 1
body = src[s:e + 1]
# hidden-loop exit: the label after the loop's back-edge branch, then the
# final phase starts at the first MFMA after it
try:
    loop_exit = next(i for i, l in enumerate(body) if re.match(r"^\.LBB\d+_31:", l.strip()))
    fin_mfma = next(i for i in range(loop_exit, len(body)) if "v_mfma" in body[i])
    fin_start = max(i for i in range(loop_exit, fin_mfma)
                    if re.match(r"^\.LBB\d+_\d+:", body[i].strip()))
except (StopIteration, ValueError):   # another kernel shape: whole-kernel patches only
    loop_exit = fin_start = len(body) - 1


def ins(op):
    return "\t" + op


new = body[:fin_start + 1]
for i in range(fin_start + 1, len(body)):
    l = body[i]
    t = l.strip()
    op = t.split()[0] if t and not t.startswith(";") else ""
    if patch == "vm0_entry" and i == fin_start + 1:
        new.append(ins("s_waitcnt vmcnt(0)"))
    if patch == "vm0_mfma" and op.startswith("v_mfma"):
        new.append(ins("s_waitcnt vmcnt(0)"))
    if patch == "vm0_load" and op.startswith("buffer_load"):
        new.append(ins("s_waitcnt vmcnt(0)"))
    if patch == "vm0_store" and op.startswith("global_store"):
        new.append(ins("s_waitcnt vmcnt(0)"))
    if patch == "bar_entry" and i == fin_start + 1:
        new += [ins("s_waitcnt vmcnt(0) lgkmcnt(0)"), ins("s_barrier")]
    if patch == "nop_accread" and op.startswith("v_accvgpr_read"):
        new += [ins("s_nop 7"), ins("s_nop 7")]
    if patch == "lgkm0_ds" and op.startswith("ds_"):
        new.append(ins("s_waitcnt lgkmcnt(0)"))
    new.append(l)
    if patch == "nop_mfma" and op.startswith("v_mfma"):
        new.append(ins("s_nop 7"))
        new.append(ins("s_nop 7"))
    if patch == "nop_load" and op.startswith("buffer_load"):
        new.append(ins("s_nop 7"))
    if patch == "lgkm0_ds" and op.startswith("ds_"):
        new.append(ins("s_waitcnt lgkmcnt(0)"))
if patch == "none":
    new = body
def mfma_srcab(t):
    ops = [x.strip() for x in t.split(None, 1)[1].split(",")]
    out = set()
    for tok in ops[1:3]:
        m = re.fullmatch(r"v\[(\d+):(\d+)\]", tok)
        if m:
            out |= set(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def load_dst(t):
    tok = t.split(None, 1)[1].split(",")[0].strip()
    m = re.fullmatch(r"v\[(\d+):(\d+)\]", tok)
    return set(range(int(m.group(1)), int(m.group(2)) + 1)) if m else set()


if patch.startswith("war_pad"):
    # war_pad<N>: before every buffer/global load whose destination overlaps
    # SrcA/SrcB of one of the last 6 MFMAs issued before it (straight-line
    # order), insert N wait states (s_nop 7 per 8)
    n = int(patch[len("war_pad"):])
    new, recent, padded = [], [], 0
    for l in body:
        t = l.strip()
        op = t.split()[0] if t and not t.startswith(";") else ""
        if re.match(r"^\.LBB\d+_\d+:", t):
            pass
        if op.startswith("v_mfma"):
            recent = (recent + [mfma_srcab(t)])[-6:]
        if op.startswith(("buffer_load", "global_load")) and " lds" not in t:
            d = load_dst(t)
            if any(d & r for r in recent):
                new += [ins("s_nop 7")] * (n // 8)
                padded += 1
        new.append(l)
    print("padded loads", padded)
def sgprs(tok):
    m = re.fullmatch(r"s\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.fullmatch(r"s(\d+)", tok)
    return {int(m.group(1))} if m else set()


def vgprs_tok(tok):
    m = re.fullmatch(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return {f"v{i}" for i in range(int(m.group(1)), int(m.group(2)) + 1)}
    return {tok} if re.fullmatch(r"v\d+", tok) else set()


if patch.startswith("nopvgpr"):
    # nopvgpr<N>: before every VALU instruction that writes a VGPR read as an
    # ADDRESS operand (voffset / vaddr) by one of the last 4 vector-memory
    # instructions, N wait states
    n = int(patch[len("nopvgpr"):])
    new, recent, hits = [], [], 0
    for l in body:
        t = l.strip()
        op = t.split()[0] if t and not t.startswith(";") else ""
        if op.startswith("v_") and not op.startswith(("v_mfma", "v_cmp", "v_readlane", "v_readfirstlane")) and " " in t:
            dst = vgprs_tok(re.split(r"[,\s]+", t.split(None, 1)[1])[0])
            if dst and any(dst & r for r in recent):
                new.append(ins(f"s_nop {n - 1}"))
                hits += 1
        if re.match(r"^\.LBB\d+_\d+:", t):
            recent = []
        new.append(l)
        if op.startswith(("buffer_", "global_")):
            toks = [x for x in re.split(r"[,\s]+", t.split(None, 1)[1]) if x]
            addr = toks[1] if ("load" in op and " lds" not in t) else toks[0]
            if op.startswith("global_store") or op.startswith("buffer_store"):
                addr = toks[0]
            recent = (recent + [vgprs_tok(addr)])[-4:]
    print("hits", hits)
if patch.startswith("nopsmov") or patch == "vm0_after_load_all":
    # nopsmov<N>: before every SALU instruction that writes an SGPR read by one
    # of the last 4 vector-memory instructions (soffset / resource), N wait
    # states; vm0_after_load_all: s_waitcnt vmcnt(0) after every VMEM load
    region = None
    if patch.startswith("nopsmov") and "_" in patch:
        patch, region = patch.split("_", 1)
    n = int(patch[len("nopsmov"):]) if patch.startswith("nopsmov") else 0
    loop_head = next((i for i, l in enumerate(body) if "Loop Header" in l), 0)
    lo, hi = {"pro": (0, loop_head - 100), "loop": (loop_head - 100, fin_start),
              "fin": (fin_start, len(body)), None: (0, len(body))}[region]
    new, recent, hits = [], [], 0
    for li, l in enumerate(body):
        t = l.strip()
        op = t.split()[0] if t and not t.startswith(";") else ""
        if op.startswith("s_") and op not in ("s_nop", "s_waitcnt", "s_barrier", "s_endpgm") \
                and not op.startswith(("s_cbranch", "s_branch")):
            dst = sgprs(t.split(None, 1)[1].split(",")[0].strip()) if " " in t else set()
            if dst and any(dst & r for r in recent) and n and lo <= li < hi:
                new.append(ins(f"s_nop {n - 1}"))
                hits += 1
        if re.match(r"^\.LBB\d+_\d+:", t):
            recent = []
        new.append(l)
        if op.startswith(("buffer_", "global_")):
            ops = [x for x in re.split(r"[,\s]+", t.split(None, 1)[1]) if x]
            rs = set()
            for tok in ops:
                rs |= sgprs(tok)
            recent = (recent + [rs])[-4:]
            if patch == "vm0_after_load_all" and "load" in op:
                new.append(ins("s_waitcnt vmcnt(0)"))
                hits += 1
    print("hits", hits)
if patch in ("vm0_mfma_all", "nop_accread_all", "vm0_hidden_exit"):
    new = []
    for i, l in enumerate(body):
        t = l.strip()
        op = t.split()[0] if t and not t.startswith(";") else ""
        if patch == "vm0_mfma_all" and op.startswith("v_mfma"):
            new.append(ins("s_waitcnt vmcnt(0)"))
        if patch == "nop_accread_all" and op.startswith("v_accvgpr_read"):
            new += [ins("s_nop 7"), ins("s_nop 7")]
        if patch == "vm0_hidden_exit" and i == loop_exit + 1:
            new.append(ins("s_waitcnt vmcnt(0) lgkmcnt(0)"))
        new.append(l)
assert patch in ("none", "vm0_entry", "vm0_mfma", "vm0_load", "vm0_store", "nop_mfma", "nop_load",
                 "bar_entry", "nop_accread", "lgkm0_ds", "vm0_mfma_all", "nop_accread_all",
                 "vm0_hidden_exit") or patch.startswith(("war_pad", "nopsmov")) \
    or patch == "vm0_after_load_all" or patch.startswith(("nopsmov", "nopvgpr")), patch
src[s:e + 1] = new
open(out_path, "w").write("\n".join(src))
print(patch, "final phase lines", fin_start, "..", len(body), "inserted", len(new) - len(body))
