"""dotdict (utils.py:20-22 of the reference)."""


class dotdict(dict):
    def __getattr__(self, name):
        try:
            return self[name]
        except KeyError as e:
            raise AttributeError(name) from e
