# round 5: round-end profile (PMC, kernel traces, bench lines) for headline, c3, c4
set -o pipefail
CONFIGS="headline c3 c4" timeout -k 10 1100 bash tools/round_profile.sh
