from .binning import BinnedMatrix, bin_matrix, compute_edges, hist_width  # noqa: F401
from .boost import TreeEnsemble, train_ensemble  # noqa: F401
from .engine import HipTreeBuilder, TreeParams  # noqa: F401
