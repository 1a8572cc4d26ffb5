"""Metrics, timing and reporting helpers."""
