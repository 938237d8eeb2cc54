# A/B of bench.py's kernel time, in-tree library vs another build, at several
# batch sizes (usage: tools/ab_bench_sizes.sh <other libsha1chunk.so> <rounds>
# <kernel> <chunks...>); runs alternate so drift hits both sides alike.
set -u
OTHER=$1; R=$2; K=$3; shift 3
mkdir -p gpurun_out/abs
for n in "$@"; do
  for i in $(seq 1 $R); do
    timeout -k 10 120 python bench.py --chunks $n --kernel $K --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/abs/new_${n}_$i.json 2>/dev/null || exit $?
    SHA1CHUNK_LIB=$OTHER timeout -k 10 120 python bench.py --chunks $n --kernel $K --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/abs/old_${n}_$i.json 2>/dev/null || exit $?
  done
done
python - "$@" <<'PY'
import json,glob,sys
for n in sys.argv[1:]:
    for side in ("new","old"):
        rs=[json.loads(open(f).read().strip().splitlines()[-1]) for f in sorted(glob.glob(f"gpurun_out/abs/{side}_{n}_*.json"))]
        ks=[r["roofline"]["kernel_ms"] for r in rs]
        print(n, side, ["%.4f"%k for k in ks], "mean %.4f"%(sum(ks)/len(ks)), "parity", all(r["parity"] for r in rs))
PY
