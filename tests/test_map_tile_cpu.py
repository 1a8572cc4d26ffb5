"""The block -> output-tile map (ops/csrc/common.h map_tile, host-compiled):
for every supertile mode the kernels use (1-5 from choose_supertile, 6 the
rotating A/B map, 0 the grouped order), every XCD sub-block shape and
batches, each block maps to exactly one in-range tile and every tile is
covered. A mis-mapping is a silent wrong result (stale tiles) or, with an
out-of-range tile, a GPU memory fault — this catches both on the CPU."""
import os
import shutil
import subprocess

import pytest

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                    "pytorch_distributed_matmul_benchmark_amd", "ops", "csrc")
HIPCC = "/opt/rocm/bin/hipcc" if os.path.exists("/opt/rocm/bin/hipcc") else shutil.which("hipcc")
pytestmark = pytest.mark.skipif(HIPCC is None, reason="hipcc not available")

PROGRAM = r"""
#include <cstdio>
#include <vector>
#include "common.h"
using namespace pdmb;
static int check(int tm_, int tn_, int batch, int st, int sub) {
  GemmArgs a{};
  a.tiles_m = tm_; a.tiles_n = tn_; a.batch = batch; a.supertile = st;
  const long long T = (long long)tm_ * tn_ * batch;
  std::vector<char> seen(T, 0);
  for (long long b = 0; b < T; ++b) {
    int bz, tm, tn;
    map_tile(a, (int)b, bz, tm, tn, sub);
    if (bz < 0 || bz >= batch || tm < 0 || tm >= tm_ || tn < 0 || tn >= tn_) {
      std::printf("OUT OF RANGE st=%d sub=%d grid=%dx%dx%d b=%lld -> %d %d %d\n", st, sub, tm_, tn_,
                  batch, b, bz, tm, tn);
      return 1;
    }
    char& s = seen[((long long)bz * tm_ + tm) * tn_ + tn];
    if (s) { std::printf("DUPLICATE st=%d sub=%d grid=%dx%dx%d b=%lld\n", st, sub, tm_, tn_, batch, b); return 1; }
    s = 1;
  }
  return 0;
}
int main() {
  const int grids[][2] = {{16, 16}, {32, 32}, {64, 64}, {64, 8}, {8, 64}, {8, 32}, {32, 8}, {4, 64},
                          {64, 4}, {4, 128}, {128, 4}, {16, 48}, {5, 7}, {3, 40}, {1, 1}, {24, 16}};
  int bad = 0, n = 0;
  for (auto& g : grids)
    for (int batch : {1, 2, 3}) {
      const int st = choose_supertile(g[0], g[1]);
      bad += check(g[0], g[1], batch, st, 0); ++n;
      bad += check(g[0], g[1], batch, 0, 0); ++n;   // grouped order
      if (st == 1) {
        for (int sub = 1; sub <= 2; ++sub) { bad += check(g[0], g[1], batch, 1, sub); ++n; }
        bad += check(g[0], g[1], batch, 6, 0); ++n;  // rotating map
      }
    }
  std::printf(bad ? "FAIL %d of %d\n" : "OK %d cases\n", bad ? bad : n, n);
  return bad != 0;
}
"""


def test_map_tile_is_a_bijection(tmp_path):
    src = tmp_path / "map_tile_check.hip"
    src.write_text(PROGRAM)
    exe = tmp_path / "map_tile_check"
    subprocess.run([HIPCC, "-O2", "-std=c++17", f"-I{CSRC}", str(src), "-o", str(exe)],
                   check=True, capture_output=True, timeout=600)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.startswith("OK"), r.stdout + r.stderr
