# The config-3b bench line with and without rocprofv3 --kernel-trace on one box
# (run under gpurun); output under gpurun_out/s3h/.
cd ${GRAFT_REPO_ROOT:-.}
R=$(pwd)
O=$R/gpurun_out/s3h
mkdir -p $O
X="--no-secondary --no-host-path --no-stream-probe --config4-objects 0 --cpu-seconds 1"
timeout -k 10 300 python3 bench.py --config cfg3b $X > $O/plain_1.json 2> $O/plain_1.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/bench.py --config cfg3b $X > $O/traced.json 2> $O/traced.err || exit $?
cd $R
timeout -k 10 300 python3 bench.py --config cfg3b $X > $O/plain_2.json 2> $O/plain_2.err || exit $?
