from dgc.horovod.compression import Compressor, Compression
from dgc.horovod.optimizer import DistributedOptimizer
