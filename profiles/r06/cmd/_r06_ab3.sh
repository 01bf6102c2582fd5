set -o pipefail
LIBS="base xc xc2" ROUNDS=3 EXPARGS="--config C2 --ntraj 1" bash scripts/gpu_evidence.sh r06/ab3_c2 ab && \
LIBS="base xc2" ROUNDS=2 bash scripts/gpu_evidence.sh r06/ab3_c3 ab && \
LIBS="xc2" ROUNDS=2 VARIANTS="GLE_NEAR3_KS=24;GLE_NEAR3_KS=64;GLE_NEAR3_KS=128;GLE_NEAR3_KS=256" bash scripts/gpu_evidence.sh r06/ab3_near ab
