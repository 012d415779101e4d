"""kdfm — MI355X-native flow-matching distillation training step (ver5) for Conformer-CTC.

Host-side mirror of the NeMo module API used by asr_train_diffm.py; all arithmetic runs in
libkdfm.so (hand-written gfx950 HIP kernels) through the C-ABI in include/kdfm.h.
"""
__version__ = "0.1.0"

import os as _os

# Kernel arguments in device memory instead of host-coherent memory: every launch's first scalar
# loads of its argument block stay on the GPU (bench step 1700 -> 1800 utt/s on the same box,
# interleaved A/B, profiles/r03/r3u_kernarg_ab.txt).  Read by the HIP runtime when it initialises,
# so it takes effect when kdfm is imported before the first HIP call; an explicit setting wins.
_os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")

