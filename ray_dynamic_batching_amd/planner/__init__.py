"""Nexus-style SLO-aware planner: squishy bin packing, rate tracking,
re-planning with minimal model moves, and the multi-model GPU scheduler."""
from .nexus import Node, Plan, Session, SquishyPlanner, assign_to_slots, count_transfers, total_transfers  # noqa
from .profiles import load_profile_csv, load_profiles, synthetic_profile, write_profile_csv  # noqa
from .rates import RateTracker  # noqa
