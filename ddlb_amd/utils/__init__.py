"""Utilities: option schema, statistics / CSV schema, roctx profiling hooks."""
