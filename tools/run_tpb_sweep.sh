mkdir -p gpurun_out/e
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/e/pytest.txt 2>&1; tail -2 gpurun_out/e/pytest.txt
for t in 256 512; do
  echo "== TPB $t"; timeout -k 10 60 python tools/step_timing2.py 3d-point-cloud-multiday-imagery_amd/libpcmkm_dbg$t.so 10 2>&1 | grep -v amdgpu.ids || exit 1
  PCM_SO=3d-point-cloud-multiday-imagery_amd/libpcmkm_t$t.so timeout -k 10 120 python bench.py --no-cpu > gpurun_out/e/b$t.txt 2>&1 || exit 1
  python -c "
import json; d=json.loads(open('gpurun_out/e/b$t.txt').read().strip().splitlines()[-1]); print('TPB $t', round(d['ms_per_step'],4), d['breakdown_ms_per_iter'], d['candidates'], d['fit'])"
done
