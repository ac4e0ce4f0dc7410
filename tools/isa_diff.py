"""Compare the device instruction streams of two `hipcc --cuda-device-only -S` outputs kernel by kernel (labels
and comments stripped): a refactor of shared device code must leave the existing kernels' ISA unchanged.
usage: python3 tools/isa_diff.py before.s after.s"""
import re
import sys


def kernels(path):
    txt = open(path).read()
    out = {}
    for m in re.finditer(r"^(_Z\w+):[^\n]*\n(.*?)^\s*s_endpgm", txt, re.S | re.M):
        body = [ln.split(";")[0].strip() for ln in m.group(2).splitlines()]
        body = [re.sub(r"\.LBB\w+", "L", ln) for ln in body if ln and not ln.startswith(".") and not ln.endswith(":")]
        out[m.group(1)] = body
    return out


def main():
    a, b = kernels(sys.argv[1]), kernels(sys.argv[2])
    same = [k for k in a if k in b and a[k] == b[k]]
    diff = [k for k in a if k in b and a[k] != b[k]]
    print(f"kernels before {len(a)} after {len(b)}: identical {len(same)}, differ {len(diff)}, "
          f"removed {len([k for k in a if k not in b])}, added {len([k for k in b if k not in a])}")
    for k in diff:
        print(f"  {k[:100]}: {len(a[k])} -> {len(b[k])} instructions")
    return 1 if diff else 0


if __name__ == "__main__":
    sys.exit(main())
