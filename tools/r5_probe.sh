set -o pipefail
mkdir -p gpurun_out
hipcc --offload-arch=gfx950 -O3 tools/kcache_probe.hip -o /tmp/kcache_probe > gpurun_out/probe_build.log 2>&1 || exit 5
timeout -k 10 120 /tmp/kcache_probe 20000 > gpurun_out/probe_dev.log 2>&1; echo "probe dev rc=$?"; cat gpurun_out/probe_dev.log
HIP_FORCE_DEV_KERNARG=0 timeout -k 10 120 /tmp/kcache_probe 20000 > gpurun_out/probe_host.log 2>&1; echo "probe host rc=$?"; cat gpurun_out/probe_host.log
bash tools/kernarg_ab.sh dev= host=HIP_FORCE_DEV_KERNARG=0 || exit 3
bash tools/gpu.sh bench20 bench1000 && cp gpurun_out/bench20.log gpurun_out/bench20_dev.log && cp gpurun_out/bench1000.log gpurun_out/bench1000_dev.log || exit 4
HIP_FORCE_DEV_KERNARG=0 bash tools/gpu.sh bench20 bench1000 prof && cp gpurun_out/bench20.log gpurun_out/bench20_host.log && cp gpurun_out/bench1000.log gpurun_out/bench1000_host.log
timeout -k 10 300 python -u tools/strong_proxy.py 4096 840 6,8 0 persistent=1,pstream_pingpong=0 4,8 > gpurun_out/proxy_pp0.log 2>&1 && \
timeout -k 10 300 python -u tools/strong_proxy.py 4096 840 6,8 0 persistent=1,pstream_pingpong=1 4,8 > gpurun_out/proxy_pp1.log 2>&1 && \
timeout -k 10 300 python -u tools/strong_proxy.py 4096 840 6,8 0 persistent=1,pstream_pingpong=0 4,8 > gpurun_out/proxy_pp0b.log 2>&1
tail -n 4 gpurun_out/proxy_pp*.log
