"""Minimal stand-in for the `attrdict` package that scripts/evaluate_model.py
imports (line 11).  The PyPI package is not installable here and is broken on
Python >= 3.10; evaluate_model.py only needs attribute access to the saved
argparse dict."""


class AttrDict(dict):
    def __getattr__(self, name):
        try:
            return self[name]
        except KeyError:
            raise AttributeError(name)

    def __setattr__(self, name, value):
        self[name] = value
