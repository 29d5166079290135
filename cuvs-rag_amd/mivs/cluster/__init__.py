"""mivs.cluster — k-means (the trainer inside ivf_flat.build)."""
from . import kmeans  # noqa: F401
