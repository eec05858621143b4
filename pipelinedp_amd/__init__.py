"""pipelinedp_amd — MI355X-native DPEngine.aggregate hot path (work in progress)."""
__version__ = "0.1.0"
