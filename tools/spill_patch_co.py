#!/usr/bin/env python3
"""Spill investigation, step 3 (profiles/r03/spill_root_cause.md): give every 128-bit store
of a code object whose data the next instruction overwrites one wait state, by moving the
s_waitcnt two instructions below it up behind the store (same bytes, no branch moves).
  python tools/spill_patch_co.py in.co out.co"""
# byte-permute each hazard site of a code object: [store][I1][I2][s_waitcnt] ->
# [store][s_waitcnt][I1][I2] (moving a wait earlier is always safe; same bytes, no branch moves)
import re, subprocess, sys
src, dst = sys.argv[1], sys.argv[2]
dis = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "-d", "--mcpu=gfx950", src], capture_output=True, text=True).stdout
ins = []
for l in dis.split("\n"):
    m = re.match(r"\s+(\S.*?)\s*//\s*([0-9A-F]+):\s*([0-9A-F ]+)$", l)
    if m: ins.append((m.group(1).strip(), int(m.group(2), 16), m.group(3).split()))
hdr = subprocess.run(["readelf", "-S", "-W", src], capture_output=True, text=True).stdout
t = [l for l in hdr.split("\n") if " .text " in l][0].split()
i_name = t.index(".text")
vaddr, foff = int(t[i_name + 2], 16), int(t[i_name + 3], 16)
data = bytearray(open(src, "rb").read())
n = 0
for i in range(len(ins) - 3):
    s, a, enc = ins[i]
    m = re.match(r"buffer_store_dwordx4 v\[(\d+):(\d+)\]", s)
    if not m: continue
    w = re.match(r"v_\S+\s+v(\d+)", ins[i + 1][0])
    if not (w and int(m.group(1)) <= int(w.group(1)) <= int(m.group(2))): continue
    i1, i2, wc = ins[i + 1], ins[i + 2], ins[i + 3]
    assert len(i1[2]) == 1 and len(i2[2]) == 1 and wc[0].startswith("s_waitcnt") and len(wc[2]) == 1, (i1, i2, wc)
    o = i1[1] - vaddr + foff
    b1, b2, b3 = data[o:o + 4], data[o + 4:o + 8], data[o + 8:o + 12]
    data[o:o + 12] = b3 + b1 + b2
    n += 1
open(dst, "wb").write(data)
print("patched", n, "sites")
