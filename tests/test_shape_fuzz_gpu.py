"""Random-shape exactness of auto (scripts/shape_fuzz.py, small sizes): every
planner path a random shape lands on — tile family, split-K, W4 / W4S, tail
forms, the padded path — returns the float64 product of small integers rounded
once to the output dtype, bit for bit."""
import importlib.util
import os
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _fuzz():
    spec = importlib.util.spec_from_file_location("shape_fuzz", os.path.join(ROOT, "scripts", "shape_fuzz.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


@pytest.mark.parametrize("seed", [11, 12])
def test_random_shapes_exact(seed, monkeypatch, capsys):
    mod = _fuzz()
    monkeypatch.setattr(sys, "argv", ["shape_fuzz.py", "--count", "8", "--seed", str(seed), "--max", "4096"])
    rc = mod.main()
    out = capsys.readouterr().out
    assert rc == 0 and '"bad": 0' in out, out[-3000:]
