set -u
mkdir -p gpurun_out
SYMBOLS=10000000 VARIANTS="default postra postmi trk default" WORKLOADS="c3 c2 frame" bash tools/ab.sh
