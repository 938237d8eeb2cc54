# round-5 study session (split phase variants, probe, verify-queue submit stats)
set -u
timeout -k 10 200 python tools/split_probe.py --lib congestion-control-with-bittorren_amd/build-ab/libsha1chunk.so --cases 97:32768,98:32768,82:32768 > gpurun_out/split_probe_r05c.log 2>&1 || exit 1
timeout -k 10 600 python tools/sweep.py --lib congestion-control-with-bittorren_amd/build-ab/libsha1chunk.so --chunks 32768 --kernels split11,split93,split81 --rounds 6 --burst 6 > gpurun_out/phase_ab_r05c.log 2>&1 || exit 1
for m in submit reserve; do SHA1CHUNK_VQ_STATS=1 timeout -k 10 120 tools/vq_zc_bench --mode $m --chunks 16384 --producers 4 --distinct 4096 >> gpurun_out/vq_stats_r05.log 2>&1 || exit 1; done
echo done
