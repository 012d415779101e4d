"""kdfm — MI355X-native flow-matching distillation training step (ver5) for Conformer-CTC.

Host-side mirror of the NeMo module API used by asr_train_diffm.py; all arithmetic runs in
libkdfm.so (hand-written gfx950 HIP kernels) through the C-ABI in include/kdfm.h.
"""
__version__ = "0.1.0"
