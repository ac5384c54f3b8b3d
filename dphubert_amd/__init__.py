"""MI355X-native DPHuBERT distill/prune training step (gfx950 HIP kernels behind a C ABI).

Public surface mirrors the reference (seas2nada/DPHuBERT):
  dphubert_amd.wav2vec2.model.wav2vec2_model(**config)
  dphubert_amd.lightning.DistillModule / DistillLoss
"""

__version__ = "0.1.0"
