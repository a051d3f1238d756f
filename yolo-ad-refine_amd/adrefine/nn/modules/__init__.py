from .conv import Conv, Conv2d, ConvTranspose2d, autopad  # noqa: F401
