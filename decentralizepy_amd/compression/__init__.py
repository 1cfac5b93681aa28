"""Payload compressors with the reference's compressor surface (compression/Compression.py)."""
