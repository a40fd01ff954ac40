# A/B builds: bash tools/ab_cmp.sh "v1 v2" "wl1 wl2"
set -u
for w in $2; do for v in $1; do bash tools/ab_env.sh $v $w "X=$v" || exit 1; done; done
