from .UGVForwardObstacleAvoidance import UGVForwardObstacleAvoidance  # noqa: F401
