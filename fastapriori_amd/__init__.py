"""fastapriori_amd — MI355X-native distributed Apriori miner and association-rule recommender.

Capabilities of relife957/FastApriori (Spark/Scala), re-designed for CDNA4:
HIP kernels for counting, RCCL (torch.distributed "nccl") for count
distribution across the GPUs of a node, a C++ host runtime for parsing,
candidate generation, rules and output.
"""
__version__ = "0.1.0"

from .models.apriori import FastApriori, MinerConfig, mine  # noqa: F401,E402
from .models.data import MiningResult, TransactionShard, Vocabulary  # noqa: F401,E402
from .models.rules import AssociationRules  # noqa: F401,E402
