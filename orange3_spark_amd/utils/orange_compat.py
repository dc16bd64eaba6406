"""Orange data model: the real ``Orange.data`` when installed, else headless stand-ins.

Orange3 is not installed in this environment (nor is Qt), so the add-on's widget logic
must be testable headlessly.  The stand-ins implement exactly the subset
the reference touches: ``Table.from_numpy(domain, X, Y, metas, W)``, ``table.X/Y/metas``,
``domain.attributes/class_vars/metas/variables`` and the three variable kinds
(reference: orangecontrib/spark/utils/data_utils.py:21-52).
"""
from __future__ import annotations

import numpy as np

try:  # pragma: no cover - exercised only where Orange is installed
    from Orange.data import ContinuousVariable, DiscreteVariable, Domain, StringVariable, Table  # noqa: F401
    HAVE_ORANGE = True
except Exception:  # noqa: BLE001
    HAVE_ORANGE = False

    class Variable:
        def __init__(self, name: str):
            self.name = name
            self.attributes = {}

        def __repr__(self):
            return f"{type(self).__name__}('{self.name}')"

        def __eq__(self, other):
            return type(self) is type(other) and self.name == other.name

        def __hash__(self):
            return hash((type(self).__name__, self.name))

        is_continuous = False
        is_discrete = False
        is_string = False
        is_primitive = True

    class ContinuousVariable(Variable):
        is_continuous = True

    class DiscreteVariable(Variable):
        is_discrete = True

        def __init__(self, name: str, values=()):
            super().__init__(name)
            self.values = list(values)

        def __repr__(self):
            return f"DiscreteVariable('{self.name}', values={self.values})"

    class StringVariable(Variable):
        is_string = True
        is_primitive = False

    class Domain:
        def __init__(self, attributes, class_vars=None, metas=None):
            self.attributes = tuple(attributes)
            if class_vars is None:
                class_vars = ()
            elif isinstance(class_vars, Variable):
                class_vars = (class_vars,)
            self.class_vars = tuple(class_vars)
            self.metas = tuple(metas or ())

        @property
        def class_var(self):
            return self.class_vars[0] if len(self.class_vars) == 1 else None

        @property
        def variables(self):
            return self.attributes + self.class_vars

        def __iter__(self):
            return iter(self.variables)

        def __len__(self):
            return len(self.variables)

        def __repr__(self):
            return f"[{', '.join(v.name for v in self.attributes)} | {', '.join(v.name for v in self.class_vars)}]"

    class Table:
        def __init__(self, domain, X, Y=None, metas=None, W=None):
            self.domain = domain
            n = X.shape[0]
            self.X = np.asarray(X, dtype=np.float64).reshape(n, len(domain.attributes))
            ncv = len(domain.class_vars)
            if Y is None or ncv == 0:
                self.Y = np.zeros((n, 0)) if ncv != 1 else np.zeros(n)
            else:
                Y = np.asarray(Y, dtype=np.float64)
                self.Y = Y.reshape(n) if ncv == 1 else Y.reshape(n, ncv)
            self.metas = np.asarray(metas, dtype=object).reshape(n, len(domain.metas)) if metas is not None \
                else np.empty((n, len(domain.metas)), dtype=object)
            self.W = np.ones(n) if W is None else np.asarray(W, dtype=np.float64)

        @classmethod
        def from_numpy(cls, domain, X, Y=None, metas=None, W=None):
            return cls(domain, X, Y, metas, W)

        def __len__(self):
            return self.X.shape[0]

        def __iter__(self):
            for i in range(len(self)):
                yield list(self.X[i]) + (list(np.atleast_1d(self.Y[i])) if self.Y.size else []) + list(self.metas[i])
