"""Word2Vec skip-gram: topical co-occurrence structure is recovered."""
import numpy as np
import pandas as pd

from h2omx.frame import Frame
from h2omx.models.word2vec import H2OWord2vecEstimator


def _corpus(n_sent=3000, seed=0):
    rng = np.random.default_rng(seed)
    topics = [[f"a{i}" for i in range(8)], [f"b{i}" for i in range(8)], [f"c{i}" for i in range(8)]]
    toks = []
    for _ in range(n_sent):
        t = topics[rng.integers(0, 3)]
        toks += list(rng.choice(t, size=rng.integers(4, 9))) + [None]
    return Frame.from_pandas(pd.DataFrame({"w": toks}))


def test_word2vec_synonyms_follow_topics():
    fr = _corpus()
    m = H2OWord2vecEstimator(vec_size=16, window_size=3, epochs=5, min_word_freq=3, seed=1,
                             init_learning_rate=0.05, sent_sample_rate=0.0).train(training_frame=fr)
    syn = m.find_synonyms("a0", 5)
    assert len(syn) == 5
    assert sum(w.startswith("a") for w in syn) >= 4, syn
    vec = m.transform(fr, aggregate_method="NONE")
    assert vec.ncols == 16 and vec.nrows == fr.nrows
    avg = m.transform(fr, aggregate_method="AVERAGE")
    assert avg.nrows == 3000
    assert m.scoring_history[-1]["training_loss"] < m.scoring_history[0]["training_loss"]
    # pre-trained import round trip
    pre = m.to_frame()
    m2 = H2OWord2vecEstimator(pre_trained=pre).train()
    assert m2.find_synonyms("b1", 3).keys() == m.find_synonyms("b1", 3).keys()
