"""Reference plugin surface (filled in below)."""
