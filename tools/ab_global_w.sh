# Config-2 A/B: the product split kernel (in-tree library) against the A/B
# build's unit 590 (W+K ring in global memory, kVGlobalW); runs alternated.
set -u
AB=congestion-control-with-bittorren_amd/build-ab/libsha1chunk.so
R=${1:-4}
mkdir -p gpurun_out/gw
for i in $(seq 1 $R); do
  timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/gw/prod_$i.json 2>/dev/null || exit $?
  SHA1CHUNK_LIB=$AB SHA1CHUNK_SPLIT_UNIT=590 timeout -k 10 120 python bench.py --kernel split --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/gw/gw_$i.json 2>/dev/null || exit $?
done
python - <<'PY'
import json,glob
for side in ("prod","gw"):
    rs=[json.loads(open(f).read().strip().splitlines()[-1]) for f in sorted(glob.glob(f"gpurun_out/gw/{side}_*.json"))]
    ks=[r["roofline"]["kernel_ms"] for r in rs]
    print(side, ["%.4f"%k for k in ks], "mean %.4f"%(sum(ks)/len(ks)), "parity", all(r["parity"] for r in rs))
PY
