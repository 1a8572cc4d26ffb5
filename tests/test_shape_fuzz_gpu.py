"""Random-shape exactness of auto (scripts/shape_fuzz.py, small sizes): every
planner path a random shape lands on — tile family, split-K, W4 / W4S, tail
forms, the padded path — returns the float64 product of small integers rounded
once to the output dtype, bit for bit."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("seed", [11, 12])
def test_random_shapes_exact(seed):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "shape_fuzz.py"), "--count", "8",
                        "--seed", str(seed), "--max", "4096"], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    assert '"bad": 0' in r.stdout
