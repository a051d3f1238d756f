import torch.nn as nn


def build_norm_layer(cfg, num_features, postfix=""):
    """GN-only restatement of mmcv.cnn.build_norm_layer as used by DyDCNv2 (reference head.py:781)."""
    cfg = dict(cfg)
    kind = cfg.pop("type")
    requires_grad = cfg.pop("requires_grad", True)
    assert kind == "GN", kind
    layer = nn.GroupNorm(num_channels=num_features, **cfg)
    for p in layer.parameters():
        p.requires_grad = requires_grad
    return "gn" + str(postfix), layer
