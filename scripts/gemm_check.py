import sys, torch
sys.path.insert(0, ".")
from h2omx.ops import dense as D
d = torch.device("cuda")
torch.manual_seed(0)
A = torch.randn(5, 6000, device=d)
Y = torch.randn(3, 5, device=d)
X = torch.randn(3, 6000, device=d)
for name, got, ref in [
    ("Y@A", D.gemm(Y, A), Y @ A),
    ("X A^T", D.gemm(X, A, tb=True), X @ A.T),
    ("X X^T", D.gemm(X, X, tb=True), X @ X.T),
    ("Y^T X", D.gemm(Y, X, ta=True), Y.T @ X),
    ("A A^T", D.gemm(A, A, tb=True), A @ A.T),
    ("Y Y^T", D.gemm(Y, Y, tb=True), Y @ Y.T),
]:
    print(name, float((got - ref).abs().max()), float(ref.abs().max()))
