#!/bin/bash
# Copy one evidence run (gpurun_out/profround_TAG, scripts/profile_r2.sh) into
# profiles/TAG under the names tests/test_bench_evidence.py and DESIGN.md cite.
#   bash scripts/collect_profiles.sh r3
TAG=${1:-r3}
S=gpurun_out/profround_$TAG
D=profiles/$TAG
mkdir -p $D/pmc_traffic
cp $S/default_bench.json $D/default_bench_under_rocprof.json
cp $S/default_trace/run_kernel_stats.csv $D/default_bench_kernel_stats.csv
[ -f $S/default_trace/run_kernel_trace.csv ] && cp $S/default_trace/run_kernel_trace.csv $D/default_bench_kernel_trace.csv
for c in cfg3b cfg2 cfg1 cfg5; do
  cp $S/${c}_bench.json $D/${c}_bench_under_rocprof.json
  cp $S/${c}_trace/run_kernel_stats.csv $D/${c}_kernel_stats.csv
done
cp $S/traffic.json $D/traffic.json
for f in $S/pmc_*/run_counter_collection.csv; do
  n=$(basename $(dirname $f)); cp $f $D/pmc_traffic/$n.csv
done
ls $D | head -40
