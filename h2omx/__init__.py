"""h2omx: an MI355X-native, H2O-compatible distributed ML cluster.

Data plane: H2O-style frames, GBM / XGBoost / DRF / GLM / K-Means /
DeepLearning / StackedEnsemble / AutoML with hand-written CDNA4 (gfx950) HIP
kernels for the hot paths and RCCL (torch.distributed "nccl") collectives over
xGMI.  Control plane: the C++ ``h2ok`` CLI and ``h2omx-operator`` in
``control/``.
"""
__version__ = "0.1.0"
