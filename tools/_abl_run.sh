cd $GRAFT_REPO_ROOT
for n in ${ABL:-0 1 3 13 15 16}; do
  if [ $n = 0 ]; then lib=leopard_amd/lib/libleopard_amd.so; else lib=leopard_amd/ablate/$n/libleopard_amd.so; fi
  echo "ablate=$n"; LEOPARD_AMD_LIB=$lib timeout -k 10 120 python tools/kbench.py 128 128 65536 128 128 1048576 2>&1 | grep -E "x "
done
