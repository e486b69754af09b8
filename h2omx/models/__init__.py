"""Model builders (H2O estimator API)."""
from .base import Model, ModelBuilder, ModelCategory  # noqa: F401
from .adaboost import H2OAdaBoostEstimator, H2ODecisionTreeEstimator  # noqa: F401
from .aggregator import H2OAggregatorEstimator  # noqa: F401
from .coxph import H2OCoxProportionalHazardsEstimator  # noqa: F401
from .deeplearning import H2ODeepLearningEstimator  # noqa: F401
from .extended_isolation_forest import H2OExtendedIsolationForestEstimator  # noqa: F401
from .ensemble import H2OStackedEnsembleEstimator  # noqa: F401
from .generic import H2OGenericEstimator  # noqa: F401
from .glm import H2OGeneralizedLinearEstimator  # noqa: F401
from .gam import H2OGeneralizedAdditiveEstimator  # noqa: F401
from .glrm import H2OGeneralizedLowRankEstimator  # noqa: F401
from .hglm import H2OHGLMEstimator  # noqa: F401
from .infogram import H2OInfogram  # noqa: F401
from .isolation_forest import H2OIsolationForestEstimator  # noqa: F401
from .isotonic import H2OIsotonicRegressionEstimator  # noqa: F401
from .kmeans import H2OKMeansEstimator  # noqa: F401
from .naive_bayes import H2ONaiveBayesEstimator  # noqa: F401
from .model_selection import H2OANOVAGLMEstimator, H2OModelSelectionEstimator  # noqa: F401
from .pca import H2OPrincipalComponentAnalysisEstimator  # noqa: F401
from .psvm import H2OSupportVectorMachineEstimator  # noqa: F401
from .rulefit import H2ORuleFitEstimator  # noqa: F401
from .svd import H2OSingularValueDecompositionEstimator  # noqa: F401
from .target_encoder import H2OTargetEncoderEstimator  # noqa: F401
from .uplift import H2OUpliftRandomForestEstimator  # noqa: F401
from .word2vec import H2OWord2vecEstimator  # noqa: F401
from .tree_models import (H2OGradientBoostingEstimator, H2ORandomForestEstimator,  # noqa: F401
                          H2OXGBoostEstimator)

ESTIMATORS = {
    "gbm": H2OGradientBoostingEstimator,
    "xgboost": H2OXGBoostEstimator,
    "drf": H2ORandomForestEstimator,
    "glm": H2OGeneralizedLinearEstimator,
    "kmeans": H2OKMeansEstimator,
    "deeplearning": H2ODeepLearningEstimator,
    "stackedensemble": H2OStackedEnsembleEstimator,
    "pca": H2OPrincipalComponentAnalysisEstimator,
    "naivebayes": H2ONaiveBayesEstimator,
    "isolationforest": H2OIsolationForestEstimator,
    "targetencoder": H2OTargetEncoderEstimator,
    "svd": H2OSingularValueDecompositionEstimator,
    "glrm": H2OGeneralizedLowRankEstimator,
    "isotonicregression": H2OIsotonicRegressionEstimator,
    "aggregator": H2OAggregatorEstimator,
    "adaboost": H2OAdaBoostEstimator,
    "decision_tree": H2ODecisionTreeEstimator,
    "extendedisolationforest": H2OExtendedIsolationForestEstimator,
    "coxph": H2OCoxProportionalHazardsEstimator,
    "rulefit": H2ORuleFitEstimator,
    "word2vec": H2OWord2vecEstimator,
    "gam": H2OGeneralizedAdditiveEstimator,
    "modelselection": H2OModelSelectionEstimator,
    "anovaglm": H2OANOVAGLMEstimator,
    "upliftdrf": H2OUpliftRandomForestEstimator,
    "infogram": H2OInfogram,
    "psvm": H2OSupportVectorMachineEstimator,
    "generic": H2OGenericEstimator,
    "hglm": H2OHGLMEstimator,
}
