"""MI355X-native hot path of Transconnectome/multimodal_neuroimage.

Layout:
  csrc/        HIP kernels for gfx950 + the C ABI (include/mmni.h) -> libmmni.so
  _lib.py      ctypes binding (fails loudly when libmmni.so is missing)
  functional   torch.autograd wrappers over the ABI
  modules/     drop-in counterparts of the reference's modules/*
  model.py     SwinTransformerV2, SwinFusion, Transformer_Net_Cross_Attention (+ 3D lifts)
  trainer.py   Trainer(sets, **kwargs) with DDP over RCCL
  data.py      synthetic volume-pair datasets / distributed sampler
"""
__version__ = "0.1.0"
