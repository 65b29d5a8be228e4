"""Drop-in replacements for the reference's `utils.*` modules used on the
hot path (anchors, box decoding / NMS, configs, pre-processing)."""
