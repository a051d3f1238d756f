"""Loss / assignment / post-processing (mirrors ultralytics/utils of the reference)."""
