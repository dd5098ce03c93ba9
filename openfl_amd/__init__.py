"""openfl_amd -- MI355X-native tensor codecs for OpenFL's compression pipelines.

The product is the Eden codec path of openfl/pipelines (randomised Hadamard
rotation + Lloyd-Max quantisation + bit-plane packing) implemented as gfx950
HIP kernels in libofl_codec.so (C ABI: include/ofl_codec.h), with the
reference's plugin surface mirrored in openfl_amd.pipelines so a plan.yaml can
select it with
    compression_pipeline:
      template: openfl_amd.pipelines.EdenPipeline
      settings: {n_bits: 8, dim_threshold: 100, device: cuda:0}
"""
__version__ = "0.1.0"

import os as _os

if _os.environ.get("OFL_HOST_KEEP_LARGE_BLOCKS") == "1":  # opt-in host-memory policy (openfl_amd/hostmem.py)
    from openfl_amd.hostmem import keep_large_blocks as _keep

    _keep()
