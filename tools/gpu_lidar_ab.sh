# k_lidar A/B (run under gpurun): the forward fans through candidate lists
# (k_lidar_fan + k_lidar_rear) vs through the BVH (MPENV_LIDAR_FAN=0,
# k_lidar), tape and combat, rocprof kernel trace + an SQ counter pass.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r04g}
OUT=gpurun_out/ab_$TAG
mkdir -p $OUT
ARGS="--steps 200 --warmup 100 --world-groups 1 --no-profile-pass --cpu-baseline off"
for act in tape combat; do
  for fan in 1 0; do
    MPENV_LIDAR_FAN=$fan timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${act}_fan$fan -o run -- \
      python3 bench.py $ARGS --actions $act > $OUT/${act}_fan$fan.json || exit 1
  done
done
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
    SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-trace --output-format csv -d $OUT/sq_tape -o run -- \
    python3 bench.py $ARGS > $OUT/sq_tape.json || exit 1
MPENV_LIDAR_FAN=0 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
    SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-trace --output-format csv -d $OUT/sq_tape_fan0 -o run -- \
    python3 bench.py $ARGS > $OUT/sq_tape_fan0.json || exit 1
python3 tools/kstats.py $OUT
