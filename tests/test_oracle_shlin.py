"""CPU: pin the sh_linearised oracle (python_work/sh_linearised.py) to the reference's own
solves (tests/golden/make_golden_shlin.py: main() run headless with a seeded generator)."""
import numpy as np

from conftest import load_golden
from oracle import shlin_oracle


def test_steps_match_reference():
    z = load_golden("shlin_steps")
    out = shlin_oracle.run(z["U0"], len(z["U"]), N=int(z["N"]), d=float(z["d"]), k=float(z["k"]),
                           r=float(z["r"]), g=float(z["g"]))
    for s, (u, ref) in enumerate(zip(out, z["U"])):
        assert np.abs(u - ref).max() <= 1e-12 * np.abs(ref).max(), s
