#!/usr/bin/env python3
"""Scan gfx950 assembly (hipcc --cuda-device-only -S) for VALU/other uses of a register whose ds_read is
still in flight: the kernels issue LDS reads as inline asm and wait for them with counted
s_waitcnt lgkmcnt(N) (DS reads complete in order), so the compiler does not know the reads are
asynchronous — a read of a pending destination, or a non-DS write to it, before the wait that covers it
is a hazard.  Straight-line over each kernel's text (branches ignored): a screening aid, not a proof.

usage: python tools/lds_hazard.py kernel.s NAME_SUBSTRING"""
import re, sys
def regs(tok):
    m = re.match(r'([va])\[(\d+):(\d+)\]', tok)
    if m: return {f"{m.group(1)}{i}" for i in range(int(m.group(2)), int(m.group(3))+1)}
    m = re.match(r'([va])(\d+)$', tok)
    if m: return {tok}
    return set()
def check(asm, fn):
    m = re.search(r'^(' + re.escape(fn) + r'):(.*?)s_endpgm', asm, re.S | re.M)
    lines = [l.strip() for l in m.group(2).split('\n') if l.strip() and not l.strip().startswith(('.', ';'))]
    pending = []  # (idx, regs)
    bad = 0
    for i, l in enumerate(lines):
        op = l.split()[0]
        if op.startswith('s_waitcnt') and 'lgkmcnt' in l:
            n = int(re.search(r'lgkmcnt\((\d+)\)', l).group(1))
            # DS ops complete in order: keep only the last n pending
            pending = pending[len(pending) - n:] if n < len(pending) else pending
            continue
        if op.startswith('s_cbranch') or op.startswith('s_branch') or op == 's_barrier':
            pass
        toks = l.replace(',', ' ').split()
        dst = regs(toks[1]) if len(toks) > 1 else set()
        srcs = set().union(*[regs(t) for t in toks[2:]]) if len(toks) > 2 else set()
        # a read of a pending destination, or a write to it, before it landed
        for j, r in pending:
            if (srcs & r) or (dst & r and not op.startswith('ds_read')):
                print("HAZARD", fn[-30:], i, l, "pending from", j, lines[j]); bad += 1
            elif dst & r and op.startswith('ds_read'):
                print("WAW-ds", i, l, "pending", lines[j])
        if op.startswith('ds_read'):
            pending.append((i, dst))
        if op in ('s_cbranch_scc0','s_cbranch_scc1','s_cbranch_vccz','s_cbranch_vccnz','s_cbranch_execz','s_cbranch_execnz','s_branch') or l.startswith('.LBB'):
            pass
    return bad
asm = open(sys.argv[1]).read()
for fn in re.findall(r'^(_Z\w*' + sys.argv[2] + r'\w*):', asm, re.M):
    print(fn, "hazards:", check(asm, fn))
