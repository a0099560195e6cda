from dgc.optim.sgd import DGCSGD
