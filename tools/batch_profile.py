"""cProfile of the batched end-to-end path (EdenPipeline.forward_batch /
backward_batch + NamedTensor build / parse, tools/e2e_bench.py 'batched'
mode) on ResNet-50 shapes."""
import cProfile
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402

from e2e_bench import run_batched, state_dict  # noqa: E402
from openfl_amd import protocols as P  # noqa: E402
from openfl_amd.pipelines import EdenPipeline  # noqa: E402
from openfl_amd.workloads import WORKLOADS  # noqa: E402

sd = state_dict(WORKLOADS[sys.argv[1] if len(sys.argv) > 1 else "resnet50_fp32"](), 100)
pipe = EdenPipeline(n_bits=8, dim_threshold=100, device="cuda:0")
for _ in range(2):
    run_batched(sd, pipe, P)
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
for _ in range(3):
    run_batched(sd, pipe, P)
pr.disable()
print(run_batched.phases)
pstats.Stats(pr).sort_stats("tottime").print_stats(22)
