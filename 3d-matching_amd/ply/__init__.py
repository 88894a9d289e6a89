from .ply import Ply

__all__ = ["Ply"]
