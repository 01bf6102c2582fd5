set -o pipefail
LIBS="base xc5 xd1 xd2 xd4 xd7" ROUNDS=3 bash scripts/gpu_evidence.sh r06/ab7_c3 ab
