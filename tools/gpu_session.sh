#!/bin/bash
# One GPU session on the gpurun box.  Every GPU step has its own time limit;
# a step that crashes, aborts or times out ends the session (nothing more
# touches the GPU); ordinary test failures (pytest rc 1) do not.
#   usage: tools/gpu_session.sh <tag> [steps...]   steps: test sweep bench prof pmc
set -u
TAG=${1:-r01}
shift || true
STEPS=${*:-"test sweep bench prof"}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
fatal() { [ "$1" -ge 124 ] || [ "$1" -eq 0 -a 1 -eq 0 ]; }

run() {  # name limit cmd...
    local name=$1 lim=$2
    shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "   rc=$rc"
    tail -n 5 "$OUT/$name.log"
    if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
        echo "FATAL step $name rc=$rc: stopping"
        exit $rc
    fi
    return 0
}

rocminfo 2>/dev/null | grep -m1 -E "gfx950" > "$OUT/arch.txt"
nproc > "$OUT/nproc.txt"; lscpu | grep -E "Model name|^CPU\(s\)" >> "$OUT/nproc.txt"

for s in $STEPS; do
    case $s in
    test)  run pytest_gpu 900 python -u -m pytest tests -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    fuzz)  SHA1CHUNK_FUZZ_SEEDS=600 run fuzz 600 python -u -m pytest tests/test_gpu_fuzz.py \
               tests/test_gpu_vq_persistent.py -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    cfg1)  run cfg1 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -s -q -p no:cacheprovider \
               -k test_config1_make_chunks_cli --timeout 200 --timeout-method thread ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    sweep) run sweep 600 python tools/sweep.py --chunks 1024,4096,16384,65536,131072 --rounds 2 --out "$OUT/sweep.json" ;;
    bench) run bench 600 python bench.py --steps 10 --warmup 2 ;;
    prof)  run rocprof 900 bash tools/profile_bench.sh $TAG ;;
    pmc)   run pmc 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- \
               python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline
           run pmc2 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- \
               python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline ;;
    mixedab) run mixedab_arrival 400 python tools/mixed_bench.py --chunks 16384,65536,131072,262144 --reps 3 \
                 --modes auto,auto@persistent --layout arrival --out "$OUT/mixedab_arrival.json"
             run mixedab_sorted 400 python tools/mixed_bench.py --chunks 65536,131072,262144 --reps 3 \
                 --modes auto,auto@persistent --layout sorted --out "$OUT/mixedab_sorted.json" ;;
    mixedsweep)
        P=""
        for h in 0 32 64 96 107 128 160 192 256 384 512; do for f in 4 8; do P="$P,plan0.$h.$f,plan0.$h.$f@persistent"; done; done
        P="auto,auto@persistent,plan1.0.0,plan1.0.0@persistent$P"
        for lay in arrival sorted; do
            run mixedsweep_$lay 500 python tools/mixed_bench.py --chunks 131072,262144 --reps 3 \
                --modes "$P" --layout $lay --out "$OUT/mixedsweep_$lay.json"
        done ;;
    pmcshape) for n in 4096 32768 131072; do run pmc_$n 700 bash tools/pmc_shape.sh "$OUT/pmc_$n" $n; done ;;
    shard) run shard32768 300 python bench.py --chunks 32768 --steps 20 --warmup 2 --no-cpu-baseline --no-latency --strong-total 0
           run cfg5 300 python tools/mixed_bench.py --chunks 16384 --reps 5 --modes auto,auto_mixedall,auto_mixedall@hw \
               --layout arrival --out "$OUT/cfg5.json" ;;
    shardab) run shardab 600 python tools/sweep.py --lib congestion-control-with-bittorren_amd/build-ab/libsha1chunk.so \
                 --chunks 32768 --kernels split11,split14,split13,split15 --rounds 5 --burst 8 --out "$OUT/shardab.json"
             run shardprod 300 python tools/sweep.py --chunks 32768,4096 --kernels split --rounds 5 --burst 8 \
                 --out "$OUT/shardprod.json" ;;
    rehearse2) SHA1_BENCH_DIST_BACKEND=gloo run rehearse2 600 python -m torch.distributed.run --nnodes=1 \
                   --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 2 ;;
    rehearse4) SHA1_BENCH_DIST_BACKEND=gloo run rehearse4 600 python -m torch.distributed.run --nnodes=1 \
                   --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 4 --steps 10 --warmup 2 ;;
    vqbench) run vqbench 600 python tools/vq_bench.py --chunks 16384 --batches 64,256,1024 --reps 3 \
                 --out "$OUT/vq_bench.json" ;;
    vqhost1) run vqhost1 300 python tools/vq_bench.py --chunks 4096 --batches 64 --reps 2 \
                 --modes host1,persistent --out "$OUT/vq_host1.json" ;;
    configs) run configs 900 python tools/bench_configs.py --out "$OUT/configs.json" ;;
    pmcicache) for n in 4096 32768; do run pmcic_$n 400 bash tools/pmc_icache.sh "$OUT/pmcic_$n" $n; done ;;
    *) echo "unknown step $s" ;;
    esac
done
echo "session done"
