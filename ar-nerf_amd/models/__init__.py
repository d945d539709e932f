"""Drop-in for the reference's `models` package (models/custom_functions.py,
models/rendering.py, models/networks.py) on the MI355X kernels."""
