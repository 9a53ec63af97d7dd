# round 3: PMC traffic per call of the GF(2^16) shapes (bench secondary / configs[3] roofline)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r03_v8; mkdir -p $OUT
rm -rf gpurun_out/pmc1 gpurun_out/pmc2
PMC_TOOL=shape_time KB_ARGS="1000,200,65536,200" bash tools/pmc.sh FETCH_SIZE WRITE_SIZE || exit 1
python3 tools/pmc_traffic.py 1000 200 65536 --loss=200 --calls=13 gpurun_out/pmc1 gpurun_out/pmc2 > $OUT/pmc_traffic_1000x200.json && cat $OUT/pmc_traffic_1000x200.json
rm -rf gpurun_out/pmc1 gpurun_out/pmc2
PMC_TOOL=shape_time KB_ARGS="32768,32768,65536,32768" bash tools/pmc.sh FETCH_SIZE WRITE_SIZE || exit 1
python3 tools/pmc_traffic.py 32768 32768 65536 --loss=32768 --calls=11 gpurun_out/pmc1 gpurun_out/pmc2 > $OUT/pmc_traffic_32768x32768.json && cat $OUT/pmc_traffic_32768x32768.json
rm -rf gpurun_out/pmc1 gpurun_out/pmc2
timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 > $OUT/bench_short.json 2> $OUT/bench_short.err || { tail -20 $OUT/bench_short.err; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/bench_short.json'))
print(json.dumps(d['sharded_object'].get('per_call'))); print(json.dumps(d['secondary'][0]['roofline']))"
