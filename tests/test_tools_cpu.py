"""The reporting tools: scaling table from sweep records / bench lines."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))

import scaling_table  # noqa: E402


def _rec(mode, ws, t, n=16384, **kw):
    r = dict(script="scaling", mode=mode, n=n, dtype="bfloat16", world_size=ws, node_tflops=t,
             max_ms=1.0, backend="native")
    r.update(kw)
    return r


def test_scaling_table_efficiency(tmp_path):
    p = tmp_path / "s.jsonl"
    recs = [_rec("independent", 1, 1400.0), _rec("independent", 2, 2800.0),
            _rec("independent", 8, 10500.0), _rec("batch_parallel", 1, 1400.0),
            _rec("batch_parallel", 8, 8400.0, overlap=True),
            _rec("independent", 1, 1300.0, backend="torch"),
            {"n": 16384, "mode": "x", "error": "boom"}]
    bench = {"metric": "m", "value": 5600.0, "n_gpus": 4, "ms_per_step": 6.0, "dtype": "bf16",
             "config": {"mode": "independent", "seq_len": 16384, "overlap": False}}
    p.write_text("\n".join(json.dumps(r) for r in recs + [bench]) + "\n")
    rows = scaling_table.table(scaling_table.load([str(p)]), size=16384)
    by = {(m, ws): (t, e) for m, n, dt, ws, t, e in rows}
    assert by[("independent", 2)] == (2800.0, 100.0)
    assert abs(by[("independent", 8)][1] - 93.75) < 1e-9
    assert ("batch_parallel+overlap", 8) in by and by[("batch_parallel+overlap", 8)][1] is None
    assert ("independent [torch]", 1) in by
    out = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "scaling_table.py"), str(p),
                          "--markdown"], capture_output=True, text=True, check=True).stdout
    assert "| independent | 16384 | bfloat16 | 8 | 10500.0 | 93.8% |" in out
