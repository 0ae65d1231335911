from .transform import ISSTestTransform  # noqa: F401
