from .synthetic import SyntheticTxSource, generate, FRAUD_RATE
from .csv_source import read_creditcard_csv

__all__ = ["SyntheticTxSource", "generate", "FRAUD_RATE", "read_creditcard_csv"]
