"""Drop-in module layer (mirrors ultralytics/nn of the reference)."""
