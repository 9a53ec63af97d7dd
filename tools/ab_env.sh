#!/bin/bash
# GPU box: bbench + kbench under each environment setting given (same library).
# usage: tools/ab_env.sh "K R B" "VAR=v ..." ["VAR=v ..."]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ARGS="$1"; shift
for cfg in "$@"; do
  echo "== $cfg"
  env $cfg timeout -k 10 120 python3 tools/bbench.py $ARGS 16 64 || exit 1
  env $cfg timeout -k 10 120 python3 tools/kbench.py $ARGS || exit 1
done
