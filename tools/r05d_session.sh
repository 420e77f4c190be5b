# round-5 session D: tests, smoke, the round profile (kernel traces, FETCH /
# WRITE / SQ passes of the fused AND separate steps), the bench line over the
# fresh PMC summary, the configs[3] profile, a world-1 mesh line
set -o pipefail
timeout -k 10 2400 bash tools/gpu_session.sh r05_d final > gpurun_out/r05_d_session.log 2>&1 || exit $?
timeout -k 10 900 bash tools/prof_config3.sh > gpurun_out/r05_d_config3.log 2>&1 || exit $?
mkdir -p gpurun_out/r05_d
timeout -k 10 400 python bench.py --multi mesh --steps 2000 --warmup 1000 --no-cpu-baseline --sweep 16 \
    > gpurun_out/r05_d/mesh_world1.json 2> gpurun_out/r05_d/mesh_world1.err
