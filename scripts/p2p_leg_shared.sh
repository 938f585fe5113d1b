set -o pipefail
mkdir -p gpurun_out/r06y
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29631 scripts/tp_leg.py 64 q4_0 1 2b 8 128 2,3 shared > gpurun_out/r06y/p2p_leg.json 2> gpurun_out/r06y/p2p_leg.err; rc=$?; echo rc=$rc; cat gpurun_out/r06y/p2p_leg.json; tail -5 gpurun_out/r06y/p2p_leg.err; exit $rc
