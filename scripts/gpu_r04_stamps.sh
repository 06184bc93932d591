cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python bench.py --no-cpu-baseline --no-c3 --no-alt-dtypes --train-epochs 0 --steps 3 --warmup 2 > gpurun_out/b_sac.json 2> gpurun_out/b_sac.err || { tail -5 gpurun_out/b_sac.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/b_sac.json')); print('SAC us/step', d['sac']['us_per_step'])"
cp mopo_amd/libmopo_hip.so /tmp/lib_keep.so && cp ab/sac_stamps.so mopo_amd/libmopo_hip.so
timeout -k 10 120 python scripts/sac_stamps.py > gpurun_out/sac_stamps.txt 2>&1
src=$?
cp /tmp/lib_keep.so mopo_amd/libmopo_hip.so
cat gpurun_out/sac_stamps.txt
exit $src
