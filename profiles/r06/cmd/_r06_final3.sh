set -o pipefail
bash scripts/gpu_evidence.sh r06/final c4shape
