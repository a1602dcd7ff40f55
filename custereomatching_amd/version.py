__version__ = "0.0.1"
