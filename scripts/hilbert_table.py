"""State table of the query order's 3-D Hilbert curve (sort.hip k_qkeys), derived from the transform itself.

sort_debug.hilbert24 (the numpy copy of sort.hip's Skilling transform) defines the order.  The curve is
self-similar: the index digit (3 bits) of a cell's octant at one level depends only on the octant and on a state
reached from the octants above it.  derive() finds the states by breadth-first search over octant prefixes, two
prefixes being the same state when the two-level digit patterns below them agree, and the table entry
state * 8 + octant = digit | next_state << 3.  check() applies the table to every 24-bit key and compares with
hilbert24 (tests/test_hilbert_table.py runs it and checks the table in sort.hip).

    python scripts/hilbert_table.py        # prints the C initialiser
"""
import os
import re
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from scripts.sort_debug import hilbert24  # noqa: E402

LEVELS = 8  # 24-bit keys: 8 octant levels, the top level in bits 21-23


def _key(prefix, suffix):
    k = 0
    for o in list(prefix) + list(suffix):
        k = (k << 3) | o
    return k << (3 * (LEVELS - len(prefix) - len(suffix)))


def _digits(prefix):
    """the two index digits below `prefix` for each of the 64 two-octant suffixes"""
    L = len(prefix)
    keys = np.array([_key(prefix, (a, b)) for a in range(8) for b in range(8)], dtype=np.uint32)
    h = hilbert24(keys)
    d0 = (h >> np.uint32(3 * (LEVELS - 1 - L))) & np.uint32(7)
    d1 = (h >> np.uint32(3 * (LEVELS - 2 - L))) & np.uint32(7)
    return tuple(int(x) for x in d0), tuple(int(x) for x in d1)


def derive():
    sig = {}
    reps = []
    todo = [()]
    sig[_digits(())] = 0
    reps.append(())
    table = {}
    while todo:
        p = todo.pop(0)
        s = sig[_digits(p)]
        d0 = _digits(p)[0]
        for o in range(8):
            q = p + (o,)
            if len(q) > LEVELS - 2:
                raise RuntimeError("state search did not close within the key's levels")
            g = _digits(q)
            if g not in sig:
                sig[g] = len(reps)
                reps.append(q)
                todo.append(q)
            table[s * 8 + o] = d0[o * 8] | (sig[g] << 3)
    return [table[i] for i in range(8 * len(reps))]


def apply(table, keys):
    keys = np.asarray(keys, dtype=np.uint32)
    tb = np.array(table, dtype=np.uint32)
    st = np.zeros_like(keys)
    h = np.zeros_like(keys)
    for L in range(LEVELS - 1, -1, -1):
        e = tb[st * np.uint32(8) + ((keys >> np.uint32(3 * L)) & np.uint32(7))]
        h = (h << np.uint32(3)) | (e & np.uint32(7))
        st = e >> np.uint32(3)
    return h


def check(table, step=1):
    keys = np.arange(0, 1 << 24, step, dtype=np.uint32)
    return bool(np.array_equal(apply(table, keys), hilbert24(keys)))


def table_in_source():
    """the initialiser of kHilbertTable in sort.hip, as a list of ints"""
    with open(os.path.join(ROOT, "mesh_amd", "csrc", "sort.hip")) as fh:
        src = fh.read()
    m = re.search(r"kHilbertTable\[\d+\]\s*=\s*\{([^}]*)\}", src)
    return [int(x, 0) for x in m.group(1).replace("\n", " ").split(",") if x.strip()]


def main():
    t = derive()
    print("// %d states; entry state * 8 + octant = digit | next state << 3" % (len(t) // 8))
    rows = [", ".join("%d" % x for x in t[i:i + 8]) for i in range(0, len(t), 8)]
    print("{" + ",\n ".join(rows) + "}")
    print("all 2^24 keys equal to hilbert24:", check(t), file=sys.stderr)


if __name__ == "__main__":
    main()
