set -o pipefail
LIBS="base xo0 xo1" ROUNDS=2 EXPARGS="--config C2 --ntraj 1" bash scripts/gpu_evidence.sh r06/ab1_c2 ab && \
LIBS="base xo1" ROUNDS=2 bash scripts/gpu_evidence.sh r06/ab1_c3 ab
