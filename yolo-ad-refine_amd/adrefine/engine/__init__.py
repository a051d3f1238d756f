"""Training-step driver (mirrors the step semantics of the reference's ultralytics/engine/trainer.py)."""
