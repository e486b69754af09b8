import os, sys, time, torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from h2omx.frame import Frame
from h2omx.frame.synthetic import wide_gaussian
from h2omx.models import H2ORandomForestEstimator
X, y = wide_gaussian(1_000_000, 100, seed=5, device="cuda")
fr = Frame.from_tensor(X, y=y, y_categorical=True)
for eng in sys.argv[1:]:
    os.environ["H2OMX_TREE_ENGINE"] = eng
    t = time.time()
    m = H2ORandomForestEstimator(ntrees=10, seed=1).train(y="response", training_frame=fr)
    torch.cuda.synchronize()
    print(eng, "DRF 10 trees depth 20:", round(time.time() - t, 2), "s  AUC", round(m.training_metrics["AUC"], 4), flush=True)
