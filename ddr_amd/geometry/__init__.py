from .trapezoidal import compute_trapezoidal_geometry

__all__ = ["compute_trapezoidal_geometry"]
