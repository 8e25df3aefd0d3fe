"""Alias of centroidalplanner_amd.pycpl (the reference's module path centroidal_planner.pycpl)."""
from centroidalplanner_amd.pycpl import *  # noqa: F401,F403
from centroidalplanner_amd.pycpl import __all__  # noqa: F401
