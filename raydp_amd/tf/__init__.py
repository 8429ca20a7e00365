"""TensorFlow estimator (reference: ``python/raydp/tf/estimator.py``).

TensorFlow has no ROCm build in this image, so ``TFEstimator`` keeps the reference's
constructor/fit surface but raises a clear ImportError when TensorFlow is missing. When a
TensorFlow install is present the estimator trains through Keras on each worker of our
trainer (``raydp_amd.train``) with ``MultiWorkerMirroredStrategy``.
"""
from raydp_amd.tf.estimator import TFEstimator

__all__ = ["TFEstimator"]
