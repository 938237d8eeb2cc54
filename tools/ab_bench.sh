# A/B of bench.py's kernel time between the in-tree library and another
# build (usage: tools/ab_bench.sh <other libsha1chunk.so> [rounds]); runs
# alternate so drift hits both sides alike.
set -u
OTHER=$1; R=${2:-4}
mkdir -p gpurun_out/ab
for i in $(seq 1 $R); do
  timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/ab/new_$i.json 2>/dev/null || exit $?
  SHA1CHUNK_LIB=$OTHER timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/ab/old_$i.json 2>/dev/null || exit $?
done
python - <<'PY'
import json,glob
for side in ("new","old"):
    ks=[json.loads(open(f).read().strip().splitlines()[-1])["roofline"]["kernel_ms"] for f in sorted(glob.glob(f"gpurun_out/ab/{side}_*.json"))]
    print(side, ["%.4f"%k for k in ks], "mean %.4f"%(sum(ks)/len(ks)))
PY
