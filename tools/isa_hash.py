#!/usr/bin/env python3
"""Per-kernel hash of the gfx950 instruction stream of a device assembly file
(hipcc --cuda-device-only -S): labels, comments, symbol names and metadata
are normalised away, so two builds compare equal exactly when every kernel's
instructions are the same.  Used to check that a source refactor leaves the
product code object unchanged (round 4: the A/B study left sha1_kernels.hip).

  python tools/isa_hash.py before.s after.s     -> per-kernel table, exit 1 on a difference
"""
import hashlib
import re
import sys


def kernels(path):
    out, name, body = {}, None, []
    for line in open(path):
        m = re.match(r"^(_Z\w+|\w+):\s*(;.*)?$", line)
        if m and not line.startswith(".") and name is None:
            name, body = m.group(1), []
            continue
        if name is not None:
            if line.startswith(".Lfunc_end"):
                out[name] = body
                name = None
                continue
            t = line.split(";")[0].strip()
            if not t or t.startswith(".") or t.endswith(":"):
                continue
            t = re.sub(r"\.LBB\d+_\d+", "L", t)
            t = re.sub(r"_Z\w+", "SYM", t)
            body.append(t)
    return out


def demangle_short(n):
    m = re.match(r"_Z\d+(\w+?)(I|v|\d)", n)
    return re.sub(r"^_Z\d+", "", n)[:60] if not m else n[:60]


def main():
    a, b = kernels(sys.argv[1]), kernels(sys.argv[2])
    ha = {k: hashlib.sha1("\n".join(v).encode()).hexdigest()[:16] for k, v in a.items()}
    hb = {k: hashlib.sha1("\n".join(v).encode()).hexdigest()[:16] for k, v in b.items()}
    # match by hash multiset (kernel names may change with a template -> plain refactor)
    same = sorted(set(ha.values()) & set(hb.values()))
    only_a = {k: h for k, h in ha.items() if h not in hb.values()}
    only_b = {k: h for k, h in hb.items() if h not in ha.values()}
    print(f"{len(ha)} functions before, {len(hb)} after, {len(same)} identical instruction streams")
    for k, h in sorted(only_a.items()):
        print(f"  only before: {h} {k} ({len(a[k])} instructions)")
    for k, h in sorted(only_b.items()):
        print(f"  only after:  {h} {k} ({len(b[k])} instructions)")
    return 1 if only_a or only_b else 0


if __name__ == "__main__":
    sys.exit(main())
