set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/gpu/r3_18.sh && bash scripts/gpu/r3_17.sh
