#!/usr/bin/env python3
"""BASELINE config #1 client half: import iris over REST into a running h2omx
cloud and train GLM binomial (versicolor vs the rest, unpenalised) and
multinomial (ridge), comparing coefficients with scikit-learn to 1e-4.

    python scripts/e2e/iris_glm_rest.py --url http://127.0.0.1:54321

Used by the ``kind-e2e`` CI job against a real (kind) cluster; the same checks
run in-process in tests/test_e2e_config1.py."""
import argparse
import os
import sys
import tempfile

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

X_COLS = ["sepal_len", "sepal_wid", "petal_len", "petal_wid"]


def main():
    from sklearn.datasets import load_iris
    from sklearn.linear_model import LogisticRegression

    from h2omx.client import H2OConnection

    ap = argparse.ArgumentParser()
    ap.add_argument("--url", default="http://127.0.0.1:54321")
    a = ap.parse_args()
    conn = H2OConnection(a.url)
    print("cloud:", conn.connect()["cloud_name"])
    d = load_iris(as_frame=True)
    df = d.frame.rename(columns=dict(zip(d.feature_names, X_COLS)))
    df["species"] = np.array(d.target_names)[d.target]
    df["versicolor"] = np.where(df.species == "versicolor", "versicolor", "other")
    df = df.drop(columns=["target"])
    with tempfile.NamedTemporaryFile("w", suffix=".csv", delete=False) as f:
        df.to_csv(f.name, index=False)
        path = f.name
    key = conn.upload_file(path, destination_frame="iris.hex")
    X = df[X_COLS].to_numpy(float)
    m = conn.train("glm", key, y="versicolor", x=X_COLS, family="binomial", **{"lambda": 0}, beta_epsilon=1e-12,
                   objective_epsilon=1e-14, max_iterations=200)
    tab = m["output"]["coefficients_table"]
    coef = dict(zip(tab["names"], tab["coefficients"]))
    sk = LogisticRegression(penalty=None, tol=1e-12, max_iter=100000).fit(X, (df.versicolor == "versicolor").astype(int))
    got = np.array([coef["Intercept"]] + [coef[c] for c in X_COLS])
    np.testing.assert_allclose(got, np.concatenate([sk.intercept_, sk.coef_[0]]), rtol=1e-4, atol=1e-4)
    print("binomial coefficients match sklearn:", got.round(5).tolist())
    n = len(df)
    m = conn.train("glm", key, y="species", x=X_COLS, family="multinomial", alpha=0.0, **{"lambda": 1.0 / n},
                   standardize=False, beta_epsilon=1e-12, objective_epsilon=1e-14, max_iterations=500)
    B = np.array(m["output"]["coefficients_table"]["coefficients"])
    B[:, 0] -= B[:, 0].mean()       # intercepts: zero-sum representative (softmax invariance)
    sk = LogisticRegression(C=1.0, tol=1e-12, max_iter=100000).fit(X, df.species.to_numpy())
    np.testing.assert_allclose(B, np.concatenate([sk.intercept_[:, None], sk.coef_], 1), rtol=1e-4, atol=1e-4)
    print("multinomial coefficients match sklearn")
    return 0


if __name__ == "__main__":
    sys.exit(main())
