cd /root/repo && mkdir -p gpurun_out && timeout -k 10 300 python -u tools/e2e_probe.py > gpurun_out/e2e_probe.txt 2>&1; grep -v amdgpu.ids gpurun_out/e2e_probe.txt
