set -o pipefail
bash scripts/r5_deep.sh r5deep4 || exit 1
for t in 1 3; do PCX_CONVN_TPS=$t NOTEST=1 bash scripts/r5_deep.sh r5deep4_tps$t || exit 1; done
