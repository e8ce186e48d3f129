"""graphconvgeo_amd -- MI355X-native graph-convolution hot path of afcarl/graphconvgeo.

Product modules (all compute runs in libgcg_spmm.so HIP kernels; no CPU fallback):
  sparse       DeviceCSR (H / X resident in HBM), spmm (= S.dot + fused epilogue)
  layers       GraphConvLayer, SparseConvolutionDenseLayer, ConvolutionDenseLayer, GCN
  distributed  1-D row partition of H + RCCL all-gather of the dense operand
  graph        H = D^-1/2 (A+I) D^-1/2 construction, host (scipy) and device (HIP)
  mentions     mention-graph parsing (host) and projection (HIP), data.py:226-375
  mlpconv      MLPCONV trainer (mlpconv.py:121-352) on the GPU
  synth        seeded synthetic graphs / features for the BASELINE configs
"""
__version__ = "0.1.0"

__all__ = ["sparse", "layers", "distributed", "graph", "mentions", "mlpconv", "synth"]
