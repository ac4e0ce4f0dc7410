"""Static instruction mix of one kernel in a hipcc device assembly file (hipcc --cuda-device-only -S):
per basic block, the counts of MFMA / VALU / SALU / LDS / VMEM instructions, the loop blocks (those
branching back to themselves or to an earlier label) first.  A design aid for the VALU budget of the
tile loops.
usage: python tools/isa_mix.py FILE.s SYMBOL_SUBSTRING [--top N] [--ops]"""
import collections
import re
import sys


def kernel_lines(path, sym):
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if l.startswith("_Z") and sym in l and l.rstrip().endswith(":")
                 or (l.startswith("_Z") and sym in l.split(":")[0] and ":" in l))
    end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
    return lines[start:end]


def classify(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith(("ds_", "buffer_load_dword_lds")):
        return "lds"
    if op.startswith(("buffer_", "global_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith(("s_waitcnt", "s_nop", "s_barrier", "s_setprio", "s_sched", "s_wait")):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("v_"):
        return "valu"
    return None


def main():
    path, sym = sys.argv[1], sys.argv[2]
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 6
    ops_detail = "--ops" in sys.argv
    blocks = []
    cur = {"label": "entry", "cnt": collections.Counter(), "ops": collections.Counter(), "back": False}
    labels = {}
    for l in kernel_lines(path, sym):
        s = l.strip()
        if re.match(r"^\.LBB\d+_\d+:", s):
            blocks.append(cur)
            cur = {"label": s[:-1], "cnt": collections.Counter(), "ops": collections.Counter(), "back": False}
            labels[s[:-1]] = len(blocks)
            continue
        if not s or s.startswith((";", ".")):
            continue
        op = s.split()[0]
        c = classify(op)
        if c is None:
            continue
        cur["cnt"][c] += 1
        cur["ops"][op] += 1
        if op.startswith("s_cbranch") or op == "s_branch":
            tgt = s.split()[-1]
            if tgt in labels or tgt == cur["label"]:
                cur["back"] = True
    blocks.append(cur)
    tot = collections.Counter()
    for b in blocks:
        tot.update(b["cnt"])
    print(f"kernel total: {dict(tot)}")
    for b in sorted(blocks, key=lambda b: -b["cnt"]["mfma"] * 100 - b["cnt"]["valu"])[:top]:
        print(f"{b['label']:>14s} {'LOOP' if b['back'] else '    '} {dict(b['cnt'])}")
        if ops_detail and b["cnt"]["mfma"]:
            for op, n in b["ops"].most_common(40):
                print(f"      {n:5d} {op}")


if __name__ == "__main__":
    main()
