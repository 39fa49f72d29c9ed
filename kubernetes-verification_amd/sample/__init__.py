from .example import paper_example  # noqa: F401
