set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05a
timeout -k 10 300 python tools/c5_probe.py --n 9 --window-log2 23 --k 32 --diags "default:0,tiled:0x100000" > gpurun_out/r05a/probe_k32.json 2> gpurun_out/r05a/probe_k32.err &&
timeout -k 10 300 python tools/c5_probe.py --n 9 --window-log2 23 --k 64 --diags "default:0" > gpurun_out/r05a/probe_k64.json 2> gpurun_out/r05a/probe_k64.err
