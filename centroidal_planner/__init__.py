"""The reference's Python package name (examples/python/test.py: ``import centroidal_planner.pycpl``):
an alias of centroidalplanner_amd's pycpl module, so code written against the reference's pybind11
module imports unchanged."""
