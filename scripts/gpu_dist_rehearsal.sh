# N>1 rehearsal on a one-GPU box: gloo process group, ranks share the GPU,
# ring state through host memory.  Sharded checksums must equal one rank's.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=${1:-dr}
C=6; S=3; W=1
timeout -k 10 200 python bench.py --checksum --frames-per-step 12 --steps $S --warmup $W > gpurun_out/${TAG}_w1.json 2> gpurun_out/${TAG}_w1.err || { echo W1 FAIL; tail gpurun_out/${TAG}_w1.err; exit 1; }
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --dist-backend gloo --checksum --frames-per-step $C --steps $S --warmup $W > gpurun_out/${TAG}_w2.json 2> gpurun_out/${TAG}_w2.err || { echo W2 FAIL; tail -20 gpurun_out/${TAG}_w2.err; exit 1; }
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29532 bench.py --gpus 2 --dist-backend gloo --frames-per-step 30 --steps 4 --warmup 1 > gpurun_out/${TAG}_w2bench.json 2> gpurun_out/${TAG}_w2bench.err || { echo W2 BENCH FAIL; tail -20 gpurun_out/${TAG}_w2bench.err; exit 1; }
python3 - $TAG <<'PY'
import json, sys
t = sys.argv[1]
def last_json(f):
    return json.loads([l for l in open(f).read().splitlines() if l.startswith('{"')][-1])
a = last_json(f"gpurun_out/{t}_w1.json"); b = last_json(f"gpurun_out/{t}_w2.json")
print("w1 frames", a["frames"], "w2 frames", b["frames"])
print("EQUAL" if a["checksums"] == b["checksums"] else "DIFFER", len(a["checksums"]))
d = last_json(f"gpurun_out/{t}_w2bench.json")
print("w2 bench", d["value"], d["n_gpus"], d["config"]["parallelism"])
PY
