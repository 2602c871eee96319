cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in base split; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03s2_$v -o b -- python3 tools/with_variant.py $v bench.py --steps 20 --warmup 2 --cpu-frames 0 --filter-frames 0 --objects 0 --hybrid-objects 0 --sustain 0 --color32 0 > gpurun_out/r03s2_$v.log 2>&1 || exit 1
python3 tools/prof_summary.py gpurun_out/r03s2_$v gpurun_out/r03s2_$v/ks.csv > /dev/null
echo "$v $(tail -1 gpurun_out/r03s2_$v.log | cut -c1-120)"
grep -h "k_batch" gpurun_out/r03s2_$v/ks.csv | cut -c1-40,100-200
done
