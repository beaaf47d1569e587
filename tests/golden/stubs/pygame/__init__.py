"""Empty pygame stand-in: the reference imports it transitively (render/__init__.py)."""
