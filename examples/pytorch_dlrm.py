"""DLRM on Criteo-shaped data (reference: examples/pytorch_dlrm.ipynb): Spark-style
preprocessing on executor processes (frequency-limited categorical vocabularies, dense ids by
frequency, log-transformed integers, random row order), then TorchEstimator training of the
MI355X-native Dlrm model (fused embedding gather + MFMA dot interaction on GPU).

There is no network here for the Kaggle Criteo file: ``CRITEO_TSV`` may point at a real
``train.txt``; otherwise a synthetic Criteo-shaped file is generated."""
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import raydp
import ray
from raydp.torch import TorchEstimator
from raydp.utils import random_split
from raydp_amd.models import dlrm_data as D
from raydp_amd.models.dlrm import Dlrm

ROWS = int(os.environ.get("DLRM_ROWS", "20000"))
EPOCHS = int(os.environ.get("DLRM_EPOCHS", "2"))

ray.init(num_cpus=8)
spark = raydp.init_spark(app_name="dlrm", num_executors=2, executor_cores=2, executor_memory="2GB")
path = os.environ.get("CRITEO_TSV")
if not path:
    path = os.path.join(tempfile.mkdtemp(), "train.txt")
    D.synthetic_criteo(path, ROWS, seed=0)
df = spark.read.schema(D.criteo_schema()).option("sep", "\t").csv(path)
df, categorical_feature_sizes = D.pre_process(df.cache(), frequency_limit="3", output_ordering="total_random",
                                              no_numeric_log_col=False)
train_df, test_df = random_split(df, [0.9, 0.1])
model = Dlrm(num_numerical_features=len(D.INT_COLS), categorical_feature_sizes=categorical_feature_sizes,
             bottom_mlp_sizes=[512, 128, 32], top_mlp_sizes=[1024, 1024, 512, 256, 1])
estimator = TorchEstimator(num_workers=int(os.environ.get("DLRM_WORKERS", "1")), model=model,
                           optimizer=torch.optim.SGD(model.parameters(), lr=0.01),
                           loss=torch.nn.BCEWithLogitsLoss(reduction="mean"),
                           feature_columns=[f"_c{i}" for i in range(1, 40)],
                           feature_types=[torch.float32] * len(D.INT_COLS) + [torch.long] * len(D.CAT_COLS),
                           label_column="_c0", label_type=torch.float, batch_size=128, num_epochs=EPOCHS)
estimator.fit_on_spark(train_df, test_df)
print([h for h in estimator.results.metrics_history if "train_loss" in h][-1])
raydp.stop_spark()
ray.shutdown()
