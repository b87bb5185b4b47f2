mkdir -p gpurun_out/r06g
timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_parity.py -k in_proj_conv_proj > gpurun_out/r06g/tests.log 2>&1 || { tail -20 gpurun_out/r06g/tests.log; exit 1; }
tail -1 gpurun_out/r06g/tests.log
timeout -k 10 120 python scripts/diag/inproj_conv_stamps.py 1 > gpurun_out/r06g/stamps.jsonl 2>&1 || { tail gpurun_out/r06g/stamps.jsonl; exit 1; }
tail -2 gpurun_out/r06g/stamps.jsonl
for i in 1 2; do timeout -k 10 120 python scripts/diag/inproj_conv_bench.py product 1 >> gpurun_out/r06g/ab.jsonl 2>&1 || exit 1; done
cat gpurun_out/r06g/ab.jsonl
for i in 1 2; do for c in 0 2; do timeout -k 10 200 python -u scripts/diag/b1_chunk_graph.py 100 in_proj_conv_clips=$c >> gpurun_out/r06g/b1.txt 2>&1 || exit 1; done; done
grep "graph replays" gpurun_out/r06g/b1.txt
