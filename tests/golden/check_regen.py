"""Regenerate fixtures with the committed make_golden.py into a temporary
directory and compare them with the committed files, member by member.

Build-container only (make_golden.py reads /root/reference).  npz files carry
zip timestamps, so the comparison is over the archive's contents: the same
member names in the same order, and every array equal in dtype, shape and
bytes.  Usage:

    python tests/golden/check_regen.py ppa_fill ppa_fill_large

prints one line per fixture and exits non-zero on the first difference.
The output of the last run is kept in profiles/r06_golden_regen.txt.
"""
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def compare(a_path, b_path):
    a, b = np.load(a_path), np.load(b_path)
    if list(a.files) != list(b.files):
        only_a = sorted(set(a.files) - set(b.files))[:5]
        only_b = sorted(set(b.files) - set(a.files))[:5]
        return f"member lists differ ({len(a.files)} vs {len(b.files)}; only committed {only_a}, only new {only_b})"
    for k in a.files:
        x, y = a[k], b[k]
        if x.dtype != y.dtype or x.shape != y.shape or x.tobytes() != y.tobytes():
            return f"member {k} differs"
    return None


def main(names):
    bad = 0
    with tempfile.TemporaryDirectory() as td:
        for name in names:
            env = dict(os.environ, OFD_GOLDEN_OUT=td)
            subprocess.run([sys.executable, os.path.join(HERE, "make_golden.py"), name], env=env, check=True,
                           stdout=subprocess.DEVNULL)
            new, old = os.path.join(td, name + ".npz"), os.path.join(HERE, name + ".npz")
            err = compare(old, new)
            n = len(np.load(old).files)
            print(f"{name}.npz: {n} members, " + ("identical to the committed file" if err is None else err))
            bad += err is not None
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:] or ["ppa_fill", "ppa_fill_large"]))
