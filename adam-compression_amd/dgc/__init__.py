"""MI355X-native Deep Gradient Compression (drop-in for emma-mens/adam-compression's ``dgc``).

Modules mirror the reference: ``dgc.memory``, ``dgc.compression``, ``dgc.horovod``,
``dgc.optim``; ``dgc.comm`` replaces ``horovod.torch`` with torch.distributed (RCCL).
"""
