import torch.nn as nn

MemoryEfficientSwish = nn.SiLU
