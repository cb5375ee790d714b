"""Instruction mix of a kernel's loops from hipcc assembly (``--cuda-device-only -S``).

Finds each backward branch (``s_cbranch_*`` / ``s_branch`` to an earlier label) inside the named
kernel and counts the instructions between the target label and the branch by class
(MFMA, VALU, exp/transcendental, cvt_pk, LDS, VMEM, SALU, waitcnt). VALU per MFMA of the hot loop
is the number the backward PMC (`profiles/r2_fa_dma_ab.md`) says bounds the FA2 backward.

    python scripts/isa_loop_mix.py fa_bwd.s 'fa_bwd_dkdv_kernel<cs336::BF16, 64, true, 0, false>'
"""

from __future__ import annotations

import re
import subprocess
import sys
from collections import Counter


def demangle(names):
    out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout
    return out.splitlines()


def kernel_body(lines, pattern):
    starts = [(i, l.split(":")[0]) for i, l in enumerate(lines) if re.match(r"^_Z\w+:", l)]
    dem = demangle([n for _, n in starts])
    for (i, _), d in zip(starts, dem):
        if pattern in d:
            j = i + 1
            while j < len(lines) and not lines[j].startswith("\t.size") and not re.match(r"^\.Lfunc_end", lines[j]):
                j += 1
            return d, lines[i:j]
    raise SystemExit(f"kernel not found: {pattern}")


def classify(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith(("v_exp", "v_log", "v_rcp", "v_rsq", "v_sqrt")):
        return "valu_trans"
    if op.startswith("v_cvt_pk"):
        return "valu_cvt_pk"
    if op.startswith(("v_accvgpr", "v_mov")):
        return "valu_mov"
    if op.startswith("v_"):
        return "valu_other"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith(("s_barrier",)):
        return "barrier"
    if op.startswith("s_"):
        return "salu"
    return None


def main():
    path, pattern = sys.argv[1], sys.argv[2]
    lines = open(path).read().splitlines()
    name, body = kernel_body(lines, pattern)
    print(name)
    labels = {l.split(":")[0]: k for k, l in enumerate(body) if re.match(r"^\.LBB\w+:", l)}
    loops = []
    for k, l in enumerate(body):
        m = re.match(r"^\s+s_c?branch\w*\s+(\.LBB\w+)", l)
        if m and m.group(1) in labels and labels[m.group(1)] < k:
            loops.append((labels[m.group(1)], k))
    for a, b in loops:
        c = Counter()
        for l in body[a:b + 1]:
            t = l.strip()
            if not t or t.startswith((".", ";")) or t.endswith(":"):
                continue
            cls = classify(t.split()[0])
            if cls:
                c[cls] += 1
        valu = sum(v for k, v in c.items() if k.startswith("valu"))
        mf = c["mfma"]
        print(f"loop lines {a}-{b}: mfma {mf}  valu {valu} ({valu / mf if mf else float('nan'):.2f}/mfma)  " + "  ".join(f"{k} {v}" for k, v in sorted(c.items())))
    if "--blocks" in sys.argv:  # per basic block (label to label) of the whole kernel, MFMA blocks only
        starts = sorted(labels.values()) + [len(body)]
        for a, b in zip(starts[:-1], starts[1:]):
            c = Counter()
            ops = Counter()
            for l in body[a:b]:
                t = l.strip()
                if not t or t.startswith((".", ";")) or t.endswith(":"):
                    continue
                cls = classify(t.split()[0])
                if cls:
                    c[cls] += 1
                    if cls.startswith("valu"):
                        ops[t.split()[0]] += 1
            if c["mfma"]:
                valu = sum(v for k, v in c.items() if k.startswith("valu"))
                print(f"  block {body[a].split(':')[0]} ({a}-{b}): mfma {c['mfma']} valu {valu} ({valu / c['mfma']:.2f}/mfma) lds {c['lds']} salu {c['salu']} | " + " ".join(f"{k} {v}" for k, v in ops.most_common(10)))


if __name__ == "__main__":
    main()
