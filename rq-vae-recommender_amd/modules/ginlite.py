"""gin-config, or the subset of it the reference configs use when gin is not installed.

`from modules.ginlite import gin` yields the real `gin` module if importable, otherwise a small
implementation of exactly what `configs/*.gin` and the reference scripts need:
``import a.b`` lines, ``scope.param = value`` bindings, values that are Python literals (ints,
floats, bools, None, quoted strings, lists) or ``%module.Enum.MEMBER`` constants registered with
``constants_from_enum``, full-line and trailing ``#`` comments; ``@configurable`` functions take
bound values as defaults (explicit call arguments win); binding a parameter the configurable does
not accept raises, as gin does (e.g. ``train.attn_dropout`` in configs/decoder_ml32m.gin:21).
"""
import ast
import functools
import importlib
import inspect


class _GinLite:
    def __init__(self):
        self._fns = {}
        self._bindings = {}
        self._constants = {}

    # -- registration
    def configurable(self, fn_or_name=None, **_):
        def register(fn, name=None):
            name = name or fn.__name__
            self._fns[name] = fn

            @functools.wraps(fn)
            def wrapper(*args, **kwargs):
                bound = dict(self._bindings.get(name, {}))
                params = list(inspect.signature(fn).parameters)
                for p in params[:len(args)]:
                    bound.pop(p, None)
                bound.update(kwargs)
                return fn(*args, **bound)
            return wrapper
        if callable(fn_or_name):
            return register(fn_or_name)
        return lambda fn: register(fn, fn_or_name)

    def constants_from_enum(self, cls=None, module=None):
        def register(c):
            mod = module or c.__module__
            for m in c:
                for key in (f"{mod}.{c.__name__}.{m.name}", f"{c.__name__}.{m.name}"):
                    self._constants[key] = m
            return c
        return register(cls) if cls is not None else register

    # -- parsing
    def _check(self, name):
        fn = self._fns.get(name)
        if fn is None:
            return
        sig = inspect.signature(fn)
        if any(p.kind == p.VAR_KEYWORD for p in sig.parameters.values()):
            return
        for param in self._bindings.get(name, {}):
            if param not in sig.parameters:
                raise ValueError(f"Configurable '{name}' doesn't have a parameter named '{param}'.")

    def _value(self, text):
        text = text.strip()
        if text.startswith("%"):
            key = text[1:]
            if key not in self._constants:
                raise ValueError(f"Unknown gin constant %{key}")
            return self._constants[key]
        return ast.literal_eval(text)

    @staticmethod
    def _strip_comment(line):
        out, quote = [], None
        for ch in line:
            if quote:
                if ch == quote:
                    quote = None
            elif ch in "\"'":
                quote = ch
            elif ch == "#":
                break
            out.append(ch)
        return "".join(out).strip()

    def parse_config(self, text):
        for raw in text.splitlines():
            line = self._strip_comment(raw)
            if not line:
                continue
            if line.startswith("import "):
                importlib.import_module(line[len("import "):].strip())
                continue
            target, _, value = line.partition("=")
            if not _:
                raise ValueError(f"Cannot parse gin line: {raw!r}")
            scope, _, param = target.strip().rpartition(".")
            self._bindings.setdefault(scope, {})[param] = self._value(value)
            self._check(scope)

    def parse_config_file(self, path):
        with open(path) as f:
            self.parse_config(f.read())

    def query_parameter(self, name):
        scope, _, param = name.rpartition(".")
        return self._bindings[scope][param]

    def clear_config(self):
        self._bindings = {}


try:  # pragma: no cover - depends on the environment
    import gin as _real_gin
    gin = _real_gin
except ImportError:
    gin = _GinLite()
