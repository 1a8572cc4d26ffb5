#!/bin/bash
# One GPU session on the box: named stages, each under its own time limit, chained so
# that the first failure (or fault / time limit) ends the session. Output per stage in
# gpurun_out/<tag>/<stage>.log (JSON results next to it); docs/REPRODUCE.md lists the
# sessions whose results are committed under profiles/.
#
#   scripts/gpu_session.sh TAG STAGE [STAGE ...] [-- NAME SECONDS COMMAND...]
#
# Stages: validate (= tests smoke bench rocprof_bench selflaunch2 selflaunch4, the
# closing pass), tests (whole GPU suite), tests_gemm / tests_fp8 / tests_signal /
# tests_overlap / tests_comm (subsets), smoke, bench (driver form), bench_quick, bench_fp8,
# native16k (pdmb_bench bf16 / fp8 at 16k), overlap_proxy, rocprof_bench, selflaunch2,
# selflaunch4, gpus2_refused (bench.py --gpus 2 on a 1-GPU box must exit 2 at once),
# ab_bf16 / ab_fp32 / ab_fp8 (auto vs hipBLASLt A/B tables), final_table (auto vs
# hipBLASLt, every dtype at 4k / 8k / 16k), reduce_bench (reduce_sum bandwidth), queue_probe (hardware-queue
# false dependencies, scripts/queue_probe.py), selflaunch8 / selflaunch8_ipc / selflaunch8_chunks
# (bench.py --gpus 8 on one GPU over gloo), mask_probe (CU-mask placement at W4S occupancy,
# runtime/cu_mask_probe), cli (every reference launcher at N = 1, --check), cli_dtypes
# (run_benchmark.sh fp16 / fp32), pmc (PMC passes: scripts/gpu_pmc.sh with
# N / KS / DT from the environment). After "--": one ad-hoc step NAME with a SECONDS limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:?tag}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  tail -6 "$OUT/$name.log"
  echo "== $name rc=$rc"
  return $rc
}
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
run_stage() {
  case "$1" in
    validate) for st in tests smoke bench rocprof_bench selflaunch2 selflaunch4; do run_stage $st || return $?; done ;;
    tests) step tests 1500 $PYT tests -m gpu ;;
    bench_fp8) step bench_fp8 400 python bench.py --dtype float8_e4m3fn --steps 20 --warmup 5 --extra-steps 5 \
                 --extra-warmup 2 && grep '^{' "$OUT/bench_fp8.log" > "$OUT/bench_fp8.json" ;;
    native16k) step native16k 400 pytorch_distributed_matmul_benchmark_amd/runtime/pdmb_bench --gpus 1 \
                 --sizes 16384 --check &&
               step native16k_fp8 400 pytorch_distributed_matmul_benchmark_amd/runtime/pdmb_bench --gpus 1 \
                 --sizes 16384 --dtype float8_e4m3fn --check ;;
    final_table) for dt in bfloat16 float16 float32 float8_e4m3fn; do
                   step final_$dt 500 python scripts/ab_kernels.py --dtype $dt --kernels auto,torch \
                     --sizes 4096 8192 16384 --rounds 5 --iters 10 || return $?
                   grep '^{' "$OUT/final_$dt.log" > "$OUT/final_$dt.jsonl"
                 done ;;
    shard_table) for dt in bfloat16 float8_e4m3fn; do
                   step shard_$dt 600 python scripts/ab_kernels.py --dtype $dt --kernels auto,torch --rounds 5 \
                     --shapes 16384,2048,16384 8192,2048,8192 8192,1024,8192 4096,2048,4096 4096,1024,4096 \
                     4096,512,4096 2048,2048,2048 || return $?
                   grep '^{' "$OUT/shard_$dt.log" > "$OUT/shard_$dt.jsonl"
                 done ;;
    pmc) (export OUT="$OUT/pmc"; mkdir -p "$OUT"; step pmc 1200 bash scripts/gpu_pmc.sh) ;;
    tests_signal) step tests_signal 600 $PYT tests/test_signal_gpu.py tests/test_overlap_gpu.py -m gpu ;;
    smoke) step smoke 180 python __graft_entry__.py smoke ;;
    bench) step bench 400 python bench.py && grep '^{' "$OUT/bench.log" > "$OUT/bench.json" ;;
    bench_quick) step bench_quick 400 python bench.py --steps 10 --warmup 3 --extra-steps 5 &&
                 grep '^{' "$OUT/bench_quick.log" > "$OUT/bench_quick.json" ;;
    overlap_proxy) step overlap_proxy 900 python scripts/overlap_proxy.py &&
                   grep '^{' "$OUT/overlap_proxy.log" > "$OUT/overlap_proxy.jsonl" ;;
    rocprof_bench) step rocprof_bench 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/rocprof" -o bench -- \
                     python3 bench.py --steps 20 --warmup 5 ;;
    selflaunch2) step selflaunch2 400 python bench.py --gpus 2 --dist-backend gloo --size 4096 --steps 3 \
                   --warmup 1 --extra-steps 2 --extra-warmup 1 ;;
    selflaunch4) step selflaunch4 400 python bench.py --gpus 4 --dist-backend gloo --size 4096 --steps 3 \
                   --warmup 1 --extra-steps 2 --extra-warmup 1 ;;
    selflaunch8) step selflaunch8 500 python bench.py --gpus 8 --dist-backend gloo --size 4096 --steps 3 \
                   --warmup 1 --extra-steps 2 --extra-warmup 1 &&
                 grep '^{' "$OUT/selflaunch8.log" > "$OUT/selflaunch8.json" ;;
    selflaunch8_ipc) step selflaunch8_ipc 500 python bench.py --gpus 8 --dist-backend gloo --size 4096 \
                       --steps 3 --warmup 1 --extra-steps 2 --extra-warmup 1 --allgather ipc --allreduce ipc &&
                     grep '^{' "$OUT/selflaunch8_ipc.log" > "$OUT/selflaunch8_ipc.json" ;;
    selflaunch8_chunks_x2) run_stage selflaunch8_chunks && cp "$OUT/selflaunch8_chunks.json" "$OUT/selflaunch8_chunks_a.json" &&
                           run_stage selflaunch8_chunks ;;
    selflaunch8_chunks) step selflaunch8_chunks 500 python bench.py --gpus 8 --dist-backend gloo --size 4096 \
                          --steps 3 --warmup 1 --extra-steps 2 --extra-warmup 1 --allgather ipc --allreduce ipc \
                          --mode matrix_parallel --overlap --chunks 2 &&
                        grep '^{' "$OUT/selflaunch8_chunks.log" > "$OUT/selflaunch8_chunks.json" ;;
    gpus2_refused) echo "== gpus2_refused"; timeout -k 10 120 python bench.py --gpus 2 > "$OUT/gpus2_refused.log" 2>&1
                   local rc=$?; cat "$OUT/gpus2_refused.log"; echo "== gpus2_refused rc=$rc (want 2)"; [ $rc -eq 2 ] ;;
    ab_bf16) step ab_bf16 900 python scripts/ab_kernels.py --dtype bfloat16 --kernels auto,torch --rounds 5 \
               --shapes 6000,6000,6100 8192,8192,1000 12345,12345,12345 6000,6000,6144 2048,2048,2049 \
               16384,16384,16384 && grep '^{' "$OUT/ab_bf16.log" > "$OUT/ab_bf16.jsonl" ;;
    ab_fp32) step ab_fp32 900 python scripts/ab_kernels.py --dtype float32 --kernels auto,f32_w4,f32_t128,torch \
               --rounds 3 --shapes 4096,2048,4096 4096,1024,4096 4096,512,4096 2048,2048,2048 6144,6144,6144 \
               8192,8192,8192 16384,16384,16384 &&
             grep '^{' "$OUT/ab_fp32.log" > "$OUT/ab_fp32.jsonl" ;;
    ab_fp32_shards) step ab_fp32_shards 900 python scripts/ab_kernels.py --dtype float32 --rounds 5 \
                      --kernels auto,f32_t128:1,f32_t128:2,f32_t128:4,f32_t128x2:1,f32_t128x2:2,f32_t128x2:4,torch \
                      --shapes 4096,512,4096 4096,1024,4096 2048,2048,2048 4096,2048,4096 8192,1024,8192 &&
                    grep '^{' "$OUT/ab_fp32_shards.log" > "$OUT/ab_fp32_shards.jsonl" ;;
    cli) step cli_basic 400 ./run_benchmark.sh 1 bfloat16 --check &&
         step cli_batch 400 ./run_scaling_benchmark.sh 1 batch_parallel bfloat16 --overlap --check &&
         step cli_matrix 400 ./run_scaling_benchmark.sh 1 matrix_parallel bfloat16 --overlap --check &&
         step cli_pipeline 400 backup/run_overlap_benchmark.sh 1 pipeline bfloat16 &&
         step cli_dp 400 backup/run_distributed_benchmark.sh 1 data_parallel bfloat16 --check &&
         step cli_fp8 400 ./run_benchmark.sh 1 float8_e4m3fn --check ;;
    cli_dtypes) step cli_fp16 400 ./run_benchmark.sh 1 float16 --check &&
                step cli_fp32 400 ./run_benchmark.sh 1 float32 --check ;;
    tests_gemm) step tests_gemm 900 $PYT tests/test_gemm_gpu.py tests/test_modes_gpu.py -m gpu ;;
    tests_overlap) step tests_overlap 900 $PYT tests/test_signal_gpu.py tests/test_overlap_gpu.py \
                     tests/test_native_bench_gpu.py tests/test_multirank_gpu.py -m gpu ;;
    ab_fp8) step ab_fp8 900 python scripts/ab_kernels.py --dtype float8_e4m3fn --kernels auto,fp8_w4,torch \
              --rounds 3 --shapes 6144,6144,6144 6000,6000,6144 7168,7168,7168 4096,4096,4096 \
              8192,2048,8192 10240,10240,10240 16384,16384,16384 &&
            grep '^{' "$OUT/ab_fp8.log" > "$OUT/ab_fp8.jsonl" ;;
    ab_fp8_tail) step ab_fp8_tail 900 python scripts/ab_kernels.py --dtype float8_e4m3fn \
                   --kernels auto,auto@PDMB_TILE_TAIL=0,auto@PDMB_TILE_TAIL=2,auto@PDMB_TILE_TAIL=4,torch \
                   --rounds 5 --shapes 6144,6144,6144 \
                   6000,6000,6144 7168,7168,7168 4608,4608,3072 10240,10240,10240 4096,4096,4096 \
                   8192,2048,8192 16384,16384,16384 &&
                 grep '^{' "$OUT/ab_fp8_tail.log" > "$OUT/ab_fp8_tail.jsonl" ;;
    ab_bf16_tail) step ab_bf16_tail 900 python scripts/ab_kernels.py --dtype bfloat16 \
                    --kernels auto,auto@PDMB_TILE_TAIL=0,auto@PDMB_TILE_TAIL=2,auto@PDMB_TILE_TAIL=4,torch \
                   --rounds 5 --shapes 6144,6144,6144 \
                    6000,6000,6144 7168,7168,7168 10000,10000,10048 10240,10240,10240 16384,16384,16384 &&
                  grep '^{' "$OUT/ab_bf16_tail.log" > "$OUT/ab_bf16_tail.jsonl" ;;
    tests_tails) step tests_tails 900 $PYT tests/test_gemm_gpu.py tests/test_fp8_gpu.py -m gpu \
                   -k "tail or tile_range" ;;
    ab_refine_fp8) step ab_refine_fp8 900 python scripts/ab_kernels.py --dtype float8_e4m3fn \
                     --kernels auto,auto@PDMB_TAIL_REFINE=0,auto@PDMB_TAIL_REFINE=2,auto@PDMB_TAIL_REFINE=4,torch \
                     --rounds 5 --shapes 6144,6144,6144 6000,6000,6144 7168,7168,7168 4608,4608,3072 \
                     10240,10240,10240 5120,5120,5120 &&
                   grep '^{' "$OUT/ab_refine_fp8.log" > "$OUT/ab_refine_fp8.jsonl" ;;
    ab_refine_bf16) step ab_refine_bf16 900 python scripts/ab_kernels.py --dtype bfloat16 \
                      --kernels auto,auto@PDMB_TAIL_REFINE=0,auto@PDMB_TAIL_REFINE=2,auto@PDMB_TAIL_REFINE=4,torch \
                      --rounds 5 --shapes 6144,6144,6144 6000,6000,6144 7168,7168,7168 10000,10000,10048 \
                      10240,10240,10240 5120,5120,5120 &&
                    grep '^{' "$OUT/ab_refine_bf16.log" > "$OUT/ab_refine_bf16.jsonl" ;;
    race_refine) step race_refine 600 env PDMB_TAIL_REFINE=4 python scripts/race_screen.py --tails --reps 50 &&
                 grep '^{' "$OUT/race_refine.log" > "$OUT/race_refine.jsonl" ;;
    tests_sk) step tests_sk 600 $PYT tests/test_fp8_gpu.py -m gpu -k "stream_k" ;;
    ab_sk) step ab_sk 900 python scripts/ab_kernels.py --dtype float8_e4m3fn \
             --kernels auto,auto@PDMB_STREAMK=1,auto@PDMB_STREAMK=2,torch --rounds 5 --shapes 5120,5120,5120 4608,4608,3072 \
             3072,3072,8192 3584,3584,4096 7168,7168,1024 6000,5888,3072 4352,4352,2048 &&
           grep '^{' "$OUT/ab_sk.log" > "$OUT/ab_sk.jsonl" ;;
    race_sk) step race_sk 600 env PDMB_STREAMK=1 python scripts/race_screen.py --tails --reps 50 &&
             grep '^{' "$OUT/race_sk.log" > "$OUT/race_sk.jsonl" ;;
    ab_fp8_onewave) step ab_fp8_onewave 900 python scripts/ab_kernels.py --dtype float8_e4m3fn \
                      --kernels auto,fp8_w4:2,fp8_w4:4,torch --rounds 5 \
                      --shapes 4096,4096,4096 8192,2048,8192 16384,2048,16384 4096,8192,4096 &&
                    grep '^{' "$OUT/ab_fp8_onewave.log" > "$OUT/ab_fp8_onewave.jsonl" ;;
    ab_dp_w4s) step ab_dp_w4s 900 python scripts/ab_kernels.py --dtype float8_e4m3fn \
                 --kernels auto,auto@PDMB_TAIL_DP_W4S=1,fp8_w4,fp8_w4s,torch --rounds 5 \
                 --shapes 4608,4608,3072 4352,4352,2048 4096,4096,4096 8192,2048,8192 5120,5120,4096 &&
               grep '^{' "$OUT/ab_dp_w4s.log" > "$OUT/ab_dp_w4s.jsonl" ;;
    ab_fp8_mid) step ab_fp8_mid 900 python scripts/ab_kernels.py --dtype float8_e4m3fn --kernels auto,fp8_w4,torch \
                  --rounds 5 --shapes 5120,5120,5120 5120,5120,4096 6144,4096,4096 4608,4608,3072 4096,4096,4096 &&
                grep '^{' "$OUT/ab_fp8_mid.log" > "$OUT/ab_fp8_mid.jsonl" ;;
    ab_refine_tile) step ab_refine_tile 900 python scripts/ab_kernels.py --dtype bfloat16 \
                      --kernels auto,auto@PDMB_TAIL_REFINE=0,torch --rounds 5 --shapes 6144,4096,4096 \
                      4608,4608,3072 3000,7000,5056 8192,3072,4096 4096,6144,4096 &&
                    grep '^{' "$OUT/ab_refine_tile.log" > "$OUT/ab_refine_tile.jsonl" ;;
    tests_f32_tail) step tests_f32_tail 600 $PYT tests/test_gemm_gpu.py -m gpu -k "f32_wave_tail" ;;
    ab_f32_tail) step ab_f32_tail 900 python scripts/ab_kernels.py --dtype float32 \
                   --kernels auto,auto@PDMB_TILE_TAIL=0,torch --rounds 3 --iters 5 --shapes 5120,5120,5120 \
                   7168,7168,7168 9216,9216,9216 3072,3072,3072 5120,5120,2048 4352,4352,4352 7168,7168,1024 &&
                 grep '^{' "$OUT/ab_f32_tail.log" > "$OUT/ab_f32_tail.jsonl" ;;
    shape_fuzz) step shape_fuzz 900 python scripts/shape_fuzz.py --count 40 --seed 1 &&
                grep '^{' "$OUT/shape_fuzz.log" > "$OUT/shape_fuzz.jsonl" ;;
    race_tails) step race_tails 600 python scripts/race_screen.py --tails --reps 50 &&
                grep '^{' "$OUT/race_tails.log" > "$OUT/race_tails.jsonl" ;;
    race) step race 600 python scripts/race_screen.py --reps 200 && grep '^{' "$OUT/race.log" > "$OUT/race.jsonl" ;;
    tests_fp8) step tests_fp8 600 $PYT tests/test_fp8_gpu.py -m gpu ;;
    tests_comm) step tests_comm 1000 $PYT tests/test_ipc_gpu.py tests/test_reduce_gpu.py \
                  tests/test_multirank_gpu.py tests/test_native_bench_gpu.py -m gpu ;;
    mask_probe) P=pytorch_distributed_matmul_benchmark_amd/runtime/cu_mask_probe
                for k in 0 8 16 32; do
                  for occ in "--threads 64 --lds 0" "--threads 256 --lds 147968"; do
                    step mask_probe_k${k}_${occ// /} 60 $P --exclude $k --blocks $((256 - k)) $occ || return $?
                    cat "$OUT/mask_probe_k${k}_${occ// /}.log" >> "$OUT/mask_probe.jsonl"
                  done
                done ;;
    peer_copy) step peer_copy 300 python scripts/peer_copy_bench.py &&
               grep '^{' "$OUT/peer_copy.log" > "$OUT/peer_copy.jsonl" ;;
    rocprof_peer_copy) step rocprof_peer_copy 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d "$OUT/rocprof_pc" -o pc -- \
                         python3 scripts/peer_copy_bench.py --arms sdma:2,kernel:32 --rounds 2 --iters 3 ;;
    mask_bits) P=pytorch_distributed_matmul_benchmark_amd/runtime/cu_mask_probe
               for b in $(seq 0 31) 64 128 192 255; do
                 step mask_bit_$b 30 $P --bits $b --blocks 256 --threads 256 --lds 147968 || return $?
                 cat "$OUT/mask_bit_$b.log" >> "$OUT/mask_bits.jsonl"
               done ;;
    queue_probe) step queue_probe 300 python scripts/queue_probe.py &&
                 grep '^{' "$OUT/queue_probe.log" > "$OUT/queue_probe.jsonl" ;;
    reduce_bench) step reduce_bench 300 python scripts/reduce_bench.py &&
                  grep '^{' "$OUT/reduce_bench.log" > "$OUT/reduce_bench.jsonl" ;;
    *) echo "unknown stage $1"; return 2 ;;
  esac
}
while [ $# -gt 0 ]; do
  if [ "$1" = "--" ]; then
    shift
    step "$@" || exit $?
    break
  fi
  run_stage "$1" || exit $?
  shift
done
echo "== session $TAG done"
