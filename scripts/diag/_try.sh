set -o pipefail
for a in "" "small_gemm_max_n=4096" "" "small_gemm_max_n=4096"; do
  timeout -k 10 180 python -u scripts/diag/b1_chunk_graph.py 50 $a 2>&1 | grep "graph replays" || exit 1
done
