# torch's own HIP runtime vs the library's (diagnostic)
mkdir -p gpurun_out
timeout -k 10 120 python -c "import torch; print('torch alone', torch.cuda.is_available(), torch.cuda.device_count())" > gpurun_out/probe_torch.log 2>&1
timeout -k 10 120 python -c "
import sys; sys.path.insert(0, 'visionx-slam_amd/python')
import vxslam, torch
c = vxslam.Context(0)
print('after vx ctx', torch.cuda.is_available(), torch.cuda.device_count())
" >> gpurun_out/probe_torch.log 2>&1
timeout -k 10 60 rocminfo 2>&1 | grep -E "Marketing|gfx" | head -4 >> gpurun_out/probe_torch.log
env | grep -E "HIP|ROCR|CUDA|HSA" >> gpurun_out/probe_torch.log
exit 0
