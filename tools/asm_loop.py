"""Compact view of a kernel's memory / barrier / MFMA instruction order from a --save-temps .s file.
Usage: python tools/asm_loop.py <file.s> <mangled kernel name> [max lines]"""
import sys

s = open(sys.argv[1]).read()
name = sys.argv[2]
i = s.index(name + ":")
j = s.index(".Lfunc_end", i)
out = []
for l in (x.strip() for x in s[i:j].splitlines()):
    if not l or l.startswith(";") or (l.startswith(".") and not l.startswith(".LBB")):
        continue
    op = l.split()[0]
    if op.startswith(("v_mfma", "s_waitcnt", "s_barrier", "global_load", "buffer_load", "ds_read", "ds_write",
                      "s_setprio", "s_cbranch", "s_branch", "global_store")) or op.startswith(".LBB"):
        out.append(l[:72])
comp, prev, cnt = [], None, 0
for l in out:
    k = l.split()[0]
    if k == prev and k.startswith(("v_mfma", "ds_read", "global_load", "ds_write", "buffer_load")):
        cnt += 1
        continue
    if prev and cnt > 1:
        comp[-1] += f"  x{cnt}"
    comp.append(l)
    prev, cnt = k, 1
if prev and cnt > 1:
    comp[-1] += f"  x{cnt}"
print("\n".join(comp[: int(sys.argv[3]) if len(sys.argv) > 3 else 150]))
