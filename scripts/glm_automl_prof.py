"""Where does the AutoML GLM (lambda_search, 3-fold CV) spend its ~2 s at
10M x 100?  cProfile of one fit on the AutoML bench's data (GPU)."""
import cProfile
import io
import pstats
import sys
import time

sys.path.insert(0, ".")
import torch  # noqa: E402

from h2omx.frame import Frame  # noqa: E402
from h2omx.frame.synthetic import wide_gaussian  # noqa: E402
from h2omx.models import H2OGeneralizedLinearEstimator  # noqa: E402

dev = torch.device("cuda", 0)
X, y = wide_gaussian(10_000_000, 100, seed=5, device=dev)
fr = Frame.from_tensor(X, y=y, y_categorical=True)
kw = dict(lambda_search=True, seed=1)
H2OGeneralizedLinearEstimator(**kw).train(y="response", training_frame=fr)   # warm-up (libraries, allocator)
torch.cuda.synchronize()
pr = cProfile.Profile()
t = time.time()
pr.enable()
m = H2OGeneralizedLinearEstimator(nfolds=3, **kw).train(y="response", training_frame=fr)
torch.cuda.synchronize()
pr.disable()
print(f"GLM lambda_search nfolds=3: {time.time() - t:.3f} s")
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(45)
print(s.getvalue())
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(25)
print(s.getvalue())
