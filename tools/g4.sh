set -o pipefail
export TMPDIR=/tmp
bash tools/lat_pmc.sh flow-hash lat || exit 1
bash tools/lat_pmc.sh xdp-counter lat || exit 1
