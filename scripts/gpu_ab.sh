cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out/ab1
timeout -k 10 300 python -u scripts/ab_dds.py 3 10 > gpurun_out/ab1/ab_dds.log 2>&1; echo "ab_dds rc=$?"
grep -v amdgpu.ids gpurun_out/ab1/ab_dds.log | tail -60
timeout -k 10 300 python -u scripts/ab_interp.py 3 10 > gpurun_out/ab1/ab_interp.log 2>&1; echo "ab_interp rc=$?"
grep -v amdgpu.ids gpurun_out/ab1/ab_interp.log | tail -40
