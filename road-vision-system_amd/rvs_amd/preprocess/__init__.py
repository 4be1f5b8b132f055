from .pipeline import PreprocessPipeline

__all__ = ["PreprocessPipeline"]
