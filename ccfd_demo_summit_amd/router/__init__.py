"""Router (Camel/Drools replacement): rule sets + scored-batch routing + response signalling."""
from .router import Router
from .rules import Rule, RuleError, RuleSet

__all__ = ["Router", "Rule", "RuleError", "RuleSet"]
