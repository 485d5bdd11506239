"""Model plugins, loaded by architecture name: models.<architecture>.Model(args, device)
(reference plugin loader: src/main.py:799-812)."""
