"""graphconvgeo_amd -- MI355X-native graph-convolution hot path of afcarl/graphconvgeo.

Product modules (all compute runs in libgcg_spmm.so HIP kernels; no CPU fallback):
  sparse       DeviceCSR (H / X resident in HBM), spmm (= S.dot + fused epilogue)
  layers       GraphConvLayer, SparseConvolutionDenseLayer, ConvolutionDenseLayer, GCN
  ops          the hot path as torch.ops.gcg.* custom ops with fake kernels (torch.compile)
  dense        output layer on the MFMA cores: f32 GEMMs, fused projection + softmax + CE
  distributed  1-D row partition of H + RCCL all-gather / halo exchange of the dense operand
  dist_train   the row-partitioned GCN training step (backward through H's symmetry)
  graph        H = D^-1/2 (A+I) D^-1/2 construction, host (scipy) and device (HIP)
  mentions     mention-graph parsing (host) and projection (HIP), data.py:226-375
  mlpconv      MLPCONV trainer (mlpconv.py:121-352) on the GPU
  synth        seeded synthetic graphs / features for the BASELINE configs
"""
import os as _os

__version__ = "0.1.0"

# A captured training step (mlpconv use_graph) has parallel branches: the side-stream weight and
# bias gradients beside the main-stream chain. The HIP runtime replays such branches on this many
# streams (read once, when HIP initialises -- hence here, before any torch.cuda call). Its default
# serialises the branches and the graph ran 2-4 % behind eager; with 8 the World step replays at
# eager's speed (profiles/r06/graph_queues_ab*.txt, tools/gpu/graph_queues.sh). Eager launches
# are unaffected; an explicit setting wins.
_os.environ.setdefault("DEBUG_HIP_FORCE_GRAPH_QUEUES", "8")

__all__ = ["sparse", "ops", "layers", "dense", "distributed", "dist_train", "graph", "mentions",
           "mlpconv", "synth"]
