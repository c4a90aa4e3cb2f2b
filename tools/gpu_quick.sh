set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02a
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02a/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r02a/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r02a/b20.json 2> gpurun_out/r02a/b20.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/r02a/b20.json'));print('s20',d['ms_per_step'],d['kernel_ms']['avg'],d['roofline']['frac'])"
timeout -k 10 200 python bench.py --gpus 1 --no-cpu-baseline > gpurun_out/r02a/b200.json 2> gpurun_out/r02a/b200.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/r02a/b200.json'));print('s200',d['ms_per_step'],d['kernel_ms']['avg'],d['roofline']['frac'])"
