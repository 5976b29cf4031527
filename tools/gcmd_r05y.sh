# round 5: round-end profile (PMC, kernel traces, bench lines) for c2, c5
set -o pipefail
CONFIGS="c2 c5" timeout -k 10 1100 bash tools/round_profile.sh
