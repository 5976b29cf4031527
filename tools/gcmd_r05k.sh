# round 5: kernel stats with the tile-sort binning (headline, c3, c4), then the small-frame
# forward parity + A/B (gcmd_r05i.sh)
set -o pipefail
ROUND=r05k CFGS="headline c3 c4" STEPS=10 bash tools/prof_iter.sh || { echo "[prof] rc=$?"; exit 1; }
echo "[prof] ok"
bash tools/gcmd_r05i.sh
