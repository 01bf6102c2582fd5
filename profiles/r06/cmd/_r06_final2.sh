set -o pipefail
bash scripts/gpu_evidence.sh r06/final trace pmc c5 c5run
