cd $GRAFT_REPO_ROOT
for c in "16 16 64 9" "16 16 64 16" "16 16 64 1" "12 16 64 4" "20 16 64 16" "40 30 64 30" "100 100 64 100" "128 128 256 128" "129 127 64 127" "1000 200 64 200"; do
  timeout -k 5 60 python tools/probe_case.py $c 2>&1 | grep -E "case|Error|error" | tail -2
done
