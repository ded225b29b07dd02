"""Built native artefacts (see native/build.py)."""
