set -e
export TMPDIR=/tmp
OUT=gpurun_out; rm -rf $OUT/tl
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $OUT/tl -o run -- python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-dominance --no-csv --no-stream --no-sort > $OUT/tl.log 2>&1
python3 tools/prof_summary.py timeline $OUT/tl ${TL_N:-75} > $OUT/tl.txt
cat $OUT/tl.txt
