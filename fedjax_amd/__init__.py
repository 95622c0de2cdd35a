"""fedjax_amd — MI355X-native FedJAX client-update aggregation (placeholder init)."""
