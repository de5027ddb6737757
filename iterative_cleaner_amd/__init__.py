"""MI355X-native surgical RFI-cleaning loop (drop-in for iterative_cleaner's clean())."""
__version__ = "0.1.0"
