"""ttga — MI355X-native evaluation-and-evolution engine for the course-timetabling GA.

Host-side mirror of nelilepo/timetabling-ga-mpi-openmp's Problem / Solution /
ga.cpp surface over the C-ABI library libttga.so (include/ttga.h).
"""
from .instance import CONFIGS, Instance, config_instance, generate, parse_tim, read_tim, write_tim  # noqa: F401
from .rng import ParkMiller, island_seed, population_seeds, random_slots  # noqa: F401

__all__ = [
    "CONFIGS", "Instance", "config_instance", "generate", "parse_tim", "read_tim", "write_tim",
    "ParkMiller", "island_seed", "population_seeds", "random_slots",
]
