for v in main hi3 main hi3; do
  lib=leopard_amd/lib/libleopard_amd.so; [ $v = main ] || lib=leopard_amd/exp/$v/libleopard_amd.so
  echo "== $v"; LEOPARD_AMD_LIB=$lib KB_SETS=1 KB_N=10 KB_WARM=3 timeout -k 10 200 python3 tools/kbench.py 32768 32768 65536 2>&1 | grep -E " x " || exit 1
done
