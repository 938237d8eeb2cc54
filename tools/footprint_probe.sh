set -u
mkdir -p gpurun_out/fp
for L in 524288 262144 131072 65536 16384; do
  timeout -k 10 120 python bench.py --chunks 131072 --chunk-len $L --kernel fused --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/fp/f_$L.json 2>/dev/null || exit $?
done
python - <<'PY'
import json
for L in (524288,262144,131072,65536,16384):
    r=json.loads(open(f"gpurun_out/fp/f_{L}.json").read().strip().splitlines()[-1])
    blocks=(L+8)//64+1
    print(L, "kernel_ms %.3f"%r["roofline"]["kernel_ms"], "us/block %.4f"%(r["roofline"]["kernel_ms"]*1e3/blocks), "GB/s %.0f"%r["roofline"]["achieved"])
PY
