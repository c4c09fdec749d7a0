# The default bench command with the product library and with an alternate
# build of it (HDX_LIB_PATH) whose config-3b kernel loads without the
# non-temporal bit, alternated twice on one box (run under gpurun); the lines
# land in gpurun_out/s2v/.
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/${AB_TAG:-s2v}
mkdir -p $O
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --cpu-seconds 2 > $O/nt_$r.log 2> $O/nt_$r.err || exit $?
  HDX_LIB_PATH=hyperdex_amd/libhdxhash_nont.so timeout -k 10 300 python -u bench.py --cpu-seconds 2 > $O/nont_$r.log 2> $O/nont_$r.err || exit $?
done
