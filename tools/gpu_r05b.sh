set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05b; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_lag_shapes.py tests/test_shard_ref.py -m gpu -x -v --timeout 300 --timeout-method thread -k "windows or shard or argument" > $O/tests.log 2>&1 &&
timeout -k 10 300 python tools/c5_probe.py --n 9 --window-log2 23 --k 32 --diags "default:0" > $O/probe_k32.json 2> $O/probe_k32.err &&
timeout -k 10 300 python tools/c5_probe.py --n 9 --window-log2 23 --k 64 --diags "default:0" > $O/probe_k64.json 2> $O/probe_k64.err
