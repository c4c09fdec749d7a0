#!/bin/bash
# micro-benchmarks (run under gpurun): CityHash loop cost, long-string loads
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
O=gpurun_out/micro; mkdir -p $O
timeout -k 10 120 tools/citybench > $O/citybench.jsonl 2> $O/citybench.err || { cat $O/citybench.err; exit 1; }
cat $O/citybench.jsonl
timeout -k 10 200 tools/lwbench 30000000 > $O/lwbench.jsonl 2> $O/lwbench.err || { cat $O/lwbench.err; exit 1; }
cat $O/lwbench.jsonl
