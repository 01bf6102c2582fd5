set -o pipefail
bash scripts/gpu_evidence.sh r06/final tests lines c1 rehearse_share noiseshare
